#!/bin/bash
# one-bracket tied re-rank after the readlane walk + key-carrying std::sort finish: tie tests, stage stamps
# (NPS_TIMING build), per-call latency against the round's earlier library
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/${1:-r04l}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ties.py tests/test_gpu_promote.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
HBX_LIB_PATH=ab/libhbx_nps.so timeout -k 10 120 python -u tools/nps_stamps.py > $OUT/stamps.txt 2>&1 || { tail -5 $OUT/stamps.txt; exit 2; }
grep distinct $OUT/stamps.txt
for L in ab/libhbx_base.so hpbandster_amd/_lib/libhbx.so; do
  echo "== $L"
  HBX_LIB_PATH=$L timeout -k 10 120 python -u tools/tie_latency.py 1000 200 2>&1 | grep distinct || exit 3
done
