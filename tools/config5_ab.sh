#!/bin/bash
# A/B of libhbx variants on config #5's lines (promotion + refit of every bracket) on ONE box, alternating:
#   bash tools/config5_ab.sh <outdir> <name>...   (via gpurun; ab/libhbx_<name>.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
cd $R
run() {
  timeout -k 10 120 python -u -c "
import json, torch, bench
print(json.dumps(bench.config5(torch.device('cuda', 0))))" > $OUT/$1 2>> $OUT/err.log
}
for i in 1 2; do
  run base_$i.json || exit 1
  for v in "$@"; do
    HBX_LIB_PATH=$R/ab/libhbx_$v.so run ${v}_$i.json || exit 1
  done
done
python3 - $OUT <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*_?.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print("%-16s refit %.3f ms (spot check %s)  select %.1f us" % (f.split("/")[-1], d["refit_all_brackets_ms"],
          d["refit_bandwidths_spot_check"], d["ms_per_launch"] * 1e3))
PY
