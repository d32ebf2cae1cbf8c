#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-r04d}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_promote.py tests/test_gpu_ties.py tests/test_gpu_batch.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/side_lines.py promote sh_stage > $O/side.json 2> $O/side.err || { tail -20 $O/side.err; exit 2; }
tail -1 $O/side.json
