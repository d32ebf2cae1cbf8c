#!/bin/bash
# Row-tile variants: parity (test_gpu_kde.py) then bench A/B.  Run via gpurun after tools/build_rt_variant.sh.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-ab_rt}
mkdir -p $OUT
cd $R
for v in rt4 rt3; do
  HBX_LIB_PATH=$R/tools/_rt/libhbx_$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_kde.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_$v.log 2>&1 || { echo "parity $v failed"; tail -20 $OUT/pytest_$v.log; exit 1; }
  tail -1 $OUT/pytest_$v.log
done
bash tools/ab_lib.sh ${1:-ab_rt} rt2=tools/_rt/libhbx_rt2.so rt4=tools/_rt/libhbx_rt4.so rt3=tools/_rt/libhbx_rt3.so default=default rt4b=tools/_rt/libhbx_rt4.so rt2b=tools/_rt/libhbx_rt2.so
