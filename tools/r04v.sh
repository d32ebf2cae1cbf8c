#!/bin/bash
# shortlist inside the exact re-score for few candidates: parity tests, 64-candidate calls with and
# without (HBX_EXACT_SCAN), the kernel timeline
set -o pipefail
O=gpurun_out/${1:-r04v}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kde.py tests/test_gpu_batch.py tests/test_gpu_ties.py tests/test_gpu_e2e.py tests/test_gpu_fetch.py tests/test_gpu_concurrency.py tests/test_gpu_kdeei.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 1 0 1 0; do
  r=$(HBX_EXACT_SCAN=$v TAIL_SMALL=1 timeout -k 10 200 python3 -u tools/tail_timeline.py run 2>>$O/wall.err) || { tail -5 $O/wall.err; exit 2; }
  echo "scan=$v small: $r" | tee -a $O/wall.txt
done
bash tools/r04p.sh ${1:-r04v}/tl > /dev/null || exit 3
head -30 $O/tl/timeline.txt
