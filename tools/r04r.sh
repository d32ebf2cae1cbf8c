#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-r04r}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kde.py tests/test_gpu_batch.py tests/test_gpu_ties.py tests/test_gpu_dist.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 0 1 0 1; do
  r=$(HBX_OBS_SPLIT=$v timeout -k 10 200 python3 -u tools/tail_timeline.py run 2>>$O/wall.err) || { tail -5 $O/wall.err; exit 3; }
  echo "split=$v configs: $r" | tee -a $O/wall.txt
done
timeout -k 10 200 python -u tools/side_lines.py config2 > $O/c2.json 2>>$O/wall.err || exit 4
tail -1 $O/c2.json | cut -c1-400
