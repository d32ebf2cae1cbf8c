#!/bin/bash
# round-4 check set on one GPU box: every GPU parity test, the default bench line, the one-bracket
# promotion latency sweep, and the gloo 2-rank rehearsal launched as a bare `bench.py --gpus 2`
set -o pipefail
O=gpurun_out/${1:-r04a}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/ \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 2; }
timeout -k 10 120 python -u tools/promote_latency.py 81,243,1000,4096,16384 2000 > $O/promote_latency.txt 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --share-gpu --steps 5 --warmup 2 --no-cpu --no-config5 \
  > $O/gloo2.json 2> $O/gloo2.err || { tail -20 $O/gloo2.err; exit 4; }
echo r04a done
