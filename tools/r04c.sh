#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-r04c}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kde.py -k "rtol or logpdf" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/precise_probe.py > $O/precise.json 2> $O/precise.err || { tail -20 $O/precise.err; exit 2; }
cat $O/precise.json
