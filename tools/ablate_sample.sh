#!/bin/bash
# Build diagnostic ablation variants of the candidate sampler into tools/_abl_s/libhbx_sN.so.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$R/hpbandster_amd/_lib/obj
OUT=$R/tools/_abl_s
mkdir -p $OUT
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I $R/hpbandster_amd/csrc -I $R/include -Wno-unused-result -munsafe-fp-atomics -ffp-contract=off"
for k in "$@"; do
  /opt/rocm/bin/hipcc $FL -DHBX_S_ABLATE=$k -c $R/hpbandster_amd/csrc/hbx_sample.hip -o $OUT/s$k.o &
done
wait
for k in "$@"; do
  objs=$(ls $OBJ/*.o | grep -v hbx_sample)
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $OUT/libhbx_s$k.so $objs $OUT/s$k.o
done
