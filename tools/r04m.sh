#!/bin/bash
# get_config computed ahead: batch / e2e / fetch tests, then the SH-stage side lines (plain and interleaved)
set -o pipefail
O=gpurun_out/${1:-r04m}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_e2e.py tests/test_gpu_fetch.py tests/test_gpu_concurrency.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/side_lines.py sh_stage > $O/side.json 2> $O/side.err || { tail -20 $O/side.err; exit 2; }
tail -1 $O/side.json
