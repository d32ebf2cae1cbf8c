#!/bin/bash
# observation splits: acquisition parity tests, 64-candidate calls with and without splits, the bench line
set -o pipefail
O=gpurun_out/${1:-r04q}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kde.py tests/test_gpu_batch.py tests/test_gpu_ties.py tests/test_gpu_e2e.py tests/test_gpu_fetch.py tests/test_gpu_concurrency.py tests/test_gpu_dist.py tests/test_gpu_kdeei.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 0 1 0 1; do
  r=$(HBX_OBS_SPLIT=$v TAIL_SMALL=1 timeout -k 10 200 python3 -u tools/tail_timeline.py run 2>>$O/wall.err) || { tail -5 $O/wall.err; exit 2; }
  echo "split=$v small: $r" | tee -a $O/wall.txt
done
for v in 0 1; do
  r=$(HBX_OBS_SPLIT=$v timeout -k 10 200 python3 -u tools/tail_timeline.py run 2>>$O/wall.err) || { tail -5 $O/wall.err; exit 3; }
  echo "split=$v configs: $r" | tee -a $O/wall.txt
done
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 4; }
python3 -c "
import json;b=json.loads(open('$O/bench.json').read().strip().split('\n')[-1]);print(b['value'], b['roofline']['frac'], b['config2']['value'], b['config2']['scoring_launch_ms'], b['batched_acquisition']['ms_sequential'], b['batched_acquisition']['ms_batched']); print({k:(b[k].get('ms_sequential'),b[k].get('ms_batched'),b[k].get('speedup')) for k in ('sh_stage','sh_stage_interleaved')})"
