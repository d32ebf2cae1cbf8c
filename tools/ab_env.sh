#!/bin/bash
# A/B of an engine environment switch on ONE box, alternating runs of the default bench line:
#   bash tools/ab_env.sh <outdir> <VAR> <value>... [-- <bench args>]   (via gpurun)
# prints the main launch statistics and config #5's promotion / refit times per run
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
VAR=$2
shift 2
vals=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do vals+=("$1"); shift; done
[ "$1" == "--" ] && shift
mkdir -p $OUT
cd $R
for i in 1 2; do
  for v in "${vals[@]}"; do
    env $VAR=$v timeout -k 10 200 python -u bench.py --no-cpu "$@" > $OUT/${VAR}_${v}_$i.json 2>> $OUT/err.log || exit 1
  done
done
python3 - $OUT <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/*_?.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    c5 = d.get("config5") or {}
    print("%-28s launch median %.4f ms | c5 select %.1f us, refit %.3f ms (frac %.3f, spot %s)" % (
        f.split("/")[-1], d["roofline"]["launch_ms_stats"]["median"], 1e3 * c5.get("ms_per_launch", float("nan")),
        c5.get("refit_all_brackets_ms", float("nan")), (c5.get("refit_roofline") or {}).get("frac", float("nan")),
        c5.get("refit_bandwidths_spot_check")))
PY
