#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-r04e}
mkdir -p $O
R=$(pwd)
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_promote.py tests/test_gpu_ties.py tests/test_gpu_fit.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/tools/tie_latency.py 1000 100 > $R/$O/tie.log 2>&1 || { tail -5 $R/$O/tie.log; exit 1; }
cd $R
grep "distinct" $O/tie.log
cut -c1-220 $(ls $O/prof/*kernel_stats.csv | head -1) | head -8
rm -f $O/prof/*kernel_trace.csv
