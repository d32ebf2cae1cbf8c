#!/bin/bash
# rescue in the combine kernel: A/B on one box of the in-tree build (pair-kernel init + combine rescue),
# the same build with HBX_COMBINE_RESCUE=0 (a rescue launch) and the HBX_PAIR_INIT=0 variant library
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04t}
mkdir -p $OUT
cd $R
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py --no-cpu --no-config5 --steps 40 > $OUT/base_$i.json 2>> $OUT/err.log || exit 1
  HBX_COMBINE_RESCUE=0 timeout -k 10 120 python -u bench.py --no-cpu --no-config5 --steps 40 > $OUT/sep_$i.json 2>> $OUT/err.log || exit 1
  HBX_LIB_PATH=$R/ab/libhbx_noinit.so timeout -k 10 120 python -u bench.py --no-cpu --no-config5 --steps 40 > $OUT/noinit_$i.json 2>> $OUT/err.log || exit 1
done
for i in 1 2; do
  for v in base sep noinit; do
    E=""; [ $v = sep ] && E="HBX_COMBINE_RESCUE=0"; [ $v = noinit ] && E="HBX_LIB_PATH=$R/ab/libhbx_noinit.so"
    r=$(env $E TAIL_SMALL=1 timeout -k 10 200 python3 -u tools/tail_timeline.py run 2>>$OUT/err.log) || exit 2
    echo "$v small: $r" >> $OUT/wall.txt
    r=$(env $E timeout -k 10 200 python3 -u tools/tail_timeline.py run 2>>$OUT/err.log) || exit 3
    echo "$v configs: $r" >> $OUT/wall.txt
  done
done
cat $OUT/wall.txt
python3 - $OUT <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*_?.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    s = d["roofline"]["launch_ms_stats"]
    print("%-14s launch median %.4f mean %.4f step %.4f" % (f.split("/")[-1], s["median"], s["mean"], d["ms_per_step"]))
PY
