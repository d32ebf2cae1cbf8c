#!/bin/bash
# Variant of libhbx.so with another hmode row-tile count (the scoring kernel and its launcher are
# rebuilt with the same -D flags):  tools/build_rt_variant.sh <name> "<flags>" -> tools/_rt/libhbx_<name>.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$R/hpbandster_amd/_lib/obj
OUT=$R/tools/_rt
mkdir -p $OUT
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I $R/hpbandster_amd/csrc -I $R/include -Wno-unused-result -munsafe-fp-atomics -ffp-contract=off -fno-slp-vectorize"
/opt/rocm/bin/hipcc $FL $2 -c $R/hpbandster_amd/csrc/hbx_score_h.hip -o $OUT/$1_h.o &
/opt/rocm/bin/hipcc $FL $2 -c $R/hpbandster_amd/csrc/hbx_kde.hip -o $OUT/$1_k.o &
wait
objs=$(ls $OBJ/*.o | grep -v "/hbx_score_h.hip.o" | grep -v "/hbx_kde.hip.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $OUT/libhbx_$1.so $objs $OUT/$1_h.o $OUT/$1_k.o
echo $OUT/libhbx_$1.so
