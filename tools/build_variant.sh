#!/bin/bash
# Build a variant of libhbx.so with extra compile flags on one source file (A/B experiments):
#   tools/build_variant.sh <name> <source.hip> "<flags>"  ->  tools/_abl/libhbx_<name>.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$R/hpbandster_amd/_lib/obj
OUT=$R/tools/_abl
mkdir -p $OUT
SRC=$2
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I $R/hpbandster_amd/csrc -I $R/include -Wno-unused-result -munsafe-fp-atomics -ffp-contract=off -fno-slp-vectorize"
/opt/rocm/bin/hipcc $FL $3 -c $R/hpbandster_amd/csrc/$SRC -o $OUT/$1.o
objs=$(ls $OBJ/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $OUT/libhbx_$1.so $objs $OUT/$1.o -L/opt/rocm/lib -lrccl
echo $OUT/libhbx_$1.so
