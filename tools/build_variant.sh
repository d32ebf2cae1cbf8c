#!/bin/bash
# Build a variant of libhbx.so with extra compile flags on some sources (A/B experiments):
#   tools/build_variant.sh <name> <src.hip[,src2.hip...]> "<flags>"  ->  ab/libhbx_<name>.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$R/hpbandster_amd/_lib/obj
OUT=$R/tools/_abl
mkdir -p $OUT $R/ab
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I $R/hpbandster_amd/csrc -I $R/include -Wno-unused-result -munsafe-fp-atomics -ffp-contract=off"
objs=$(ls $OBJ/*.o)
vobjs=""
for SRC in ${2//,/ }; do
  /opt/rocm/bin/hipcc $FL $3 -c $R/hpbandster_amd/csrc/$SRC -o $OUT/$1_$SRC.o
  objs=$(echo "$objs" | grep -v "/$SRC.o")
  vobjs="$vobjs $OUT/$1_$SRC.o"
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $R/ab/libhbx_$1.so $objs $vobjs -L/opt/rocm/lib -lrccl
echo $R/ab/libhbx_$1.so
