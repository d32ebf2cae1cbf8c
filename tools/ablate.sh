#!/bin/bash
# Build diagnostic ablation variants of the hmode scoring kernel into tools/_abl/libhbx_ablN.so
# (the other objects are the regular build's).  Timing only: results of ablated builds are wrong.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$R/hpbandster_amd/_lib/obj
OUT=$R/tools/_abl
mkdir -p $OUT
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I $R/hpbandster_amd/csrc -I $R/include -Wno-unused-result -munsafe-fp-atomics -ffp-contract=off -fno-slp-vectorize"
for k in "$@"; do
  /opt/rocm/bin/hipcc $FL -DHBX_H_ABLATE=$k -c $R/hpbandster_amd/csrc/hbx_score_h.hip -o $OUT/h_abl$k.o &
done
wait
for k in "$@"; do
  objs=$(ls $OBJ/*.o | grep -v hbx_score_h)
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $OUT/libhbx_abl$k.so $objs $OUT/h_abl$k.o
done
ls -la $OUT
