#!/bin/bash
# fused combine: parity tests + host-path timing A/B
set -o pipefail
O=gpurun_out/${1:-r04b}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_kde.py \
  -k "fused or batch or acquire" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/host_path.py > $O/host_path.json 2> $O/host_path.err || { tail -20 $O/host_path.err; exit 2; }
cat $O/host_path.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/host_path.py --reps 50 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 3; }
cd $GRAFT_REPO_ROOT
cp $(ls $O/prof/*kernel_stats.csv | head -1) $O/kernel_stats.csv
rm -f $O/prof/*kernel_trace.csv
cut -c1-200 $O/kernel_stats.csv | head -30
