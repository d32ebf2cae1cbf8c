#!/bin/bash
# A/B of the l+g pair launch against two launches (run via gpurun after tools/gpu_check.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-ab_pair}
mkdir -p $OUT
cd $R
for i in 1 2; do
  HBX_SCORE_PAIR=0 timeout -k 10 120 python -u bench.py --no-cpu --no-config5 > $OUT/two_$i.json 2>> $OUT/err.log || exit 1
  timeout -k 10 120 python -u bench.py --no-cpu --no-config5 > $OUT/pair_$i.json 2>> $OUT/err.log || exit 1
done
python - $OUT <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*_?.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], "%.4e" % d["value"], d["roofline"]["ms_per_launch"])
PY
