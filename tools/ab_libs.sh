#!/bin/bash
# A/B of libhbx variants (ab/libhbx_<name>.so) against the in-tree build on ONE box, alternating runs:
#   bash tools/ab_libs.sh <outdir> <name>...   (via gpurun)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
cd $R
for i in 1 2; do
  timeout -k 10 120 python -u bench.py --no-cpu --no-config5 --steps 30 > $OUT/base_$i.json 2>> $OUT/err.log || exit 1
  for v in "$@"; do
    HBX_LIB_PATH=$R/ab/libhbx_$v.so timeout -k 10 120 python -u bench.py --no-cpu --no-config5 --steps 30 > $OUT/${v}_$i.json 2>> $OUT/err.log || exit 1
  done
done
python3 - $OUT <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*_?.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    s = d["roofline"]["launch_ms_stats"]
    c2 = d.get("config2", {})
    print("%-16s median %.4f mean %.4f shortlist %s step %.4f config2 step %s" % (f.split("/")[-1], s["median"], s["mean"],
          d["config"]["shortlist"], d["ms_per_step"], c2.get("ms_per_step")))
PY
