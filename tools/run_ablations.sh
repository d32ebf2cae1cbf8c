#!/bin/bash
# GPU box: scoring sweep for the regular build and each tools/_abl variant (timing only).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/abl
mkdir -p $OUT
cd $R
timeout -k 10 120 python -u tools/score_sweep.py > $OUT/base.json 2>&1 || exit 1
for f in tools/_abl/libhbx_abl*.so; do
  k=$(basename $f .so)
  HBX_LIB_PATH=$R/$f timeout -k 10 120 python -u tools/score_sweep.py > $OUT/$k.json 2>&1 || exit 2
done
echo ablations done
