#!/bin/bash
# exact re-score loads by dependency level + fence-free record publish: parity tests, then wall time per
# drop-in call (config #2 / #3) for the baseline library (ab/libhbx_base.so) and the new one, alternated,
# then the new one's kernel timeline
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/${1:-r04j}
mkdir -p $OUT
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kde.py tests/test_gpu_fetch.py tests/test_gpu_batch.py tests/test_gpu_ties.py tests/test_gpu_e2e.py tests/test_gpu_concurrency.py tests/test_gpu_dist.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do
  HBX_LIB_PATH=ab/libhbx_base.so timeout -k 10 200 python3 -u tools/tail_timeline.py run > $OUT/wall_base_$i.json 2>> $OUT/wall.err || { tail -20 $OUT/wall.err; exit 2; }
  HBX_EXACT_FINAL=0 timeout -k 10 200 python3 -u tools/tail_timeline.py run > $OUT/wall_twolaunch_$i.json 2>> $OUT/wall.err || { tail -20 $OUT/wall.err; exit 3; }
  timeout -k 10 200 python3 -u tools/tail_timeline.py run > $OUT/wall_new_$i.json 2>> $OUT/wall.err || { tail -20 $OUT/wall.err; exit 3; }
  echo "base: $(cat $OUT/wall_base_$i.json)"; echo "two launches: $(cat $OUT/wall_twolaunch_$i.json)"; echo "new:  $(cat $OUT/wall_new_$i.json)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- \
  python3 $R/tools/tail_timeline.py run > $OUT/traced.json 2> $OUT/trace.log || { tail -5 $OUT/trace.log; exit 4; }
T=$(ls $OUT/trace/*kernel_trace.csv $OUT/trace/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 $R/tools/tail_timeline.py show $T > $OUT/timeline.txt || exit 5
rm -f $T
cat $OUT/timeline.txt
