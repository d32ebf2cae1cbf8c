#!/bin/bash
# A/B of the hmode scoring kernels (16x16 default vs HBX_SCORE_TILE=32) on the bench workload.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-ab}
mkdir -p $OUT
cd $R
for t in 32 16; do
  HBX_SCORE_TILE=$t timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-config5 > $OUT/bench_t$t.json 2> $OUT/bench_t$t.err || { echo "bench t$t failed"; tail -20 $OUT/bench_t$t.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_t$t.json')); print('tile', $t, '%.3e' % d['value'], d['roofline']['ms_per_launch'], 'shortlist', d['config']['shortlist'], 'winner', d['config']['winner'])"
done
