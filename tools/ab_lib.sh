#!/bin/bash
# A/B of library builds on the bench workload: tools/ab_lib.sh <out> <name>=<lib or "default"> ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
cd $R
for spec in "$@"; do
  name=${spec%%=*}; lib=${spec#*=}
  if [ "$lib" = default ]; then unset HBX_LIB_PATH; else export HBX_LIB_PATH=$R/$lib; fi
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-config5 > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { echo "bench $name failed"; tail -20 $OUT/bench_$name.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$name.json')); print('$name', '%.3e' % d['value'], 'step %.4f' % d['ms_per_step'], d['roofline']['ms_per_launch'], 'shortlist', d['config']['shortlist'], 'winner', d['config']['winner'])"
done
