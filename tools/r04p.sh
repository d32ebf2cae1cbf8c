#!/bin/bash
# kernel timeline of 64-candidate acquisitions (get_config's default size) against 400 / 10000 observations
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/${1:-r04p}
mkdir -p $OUT
export TAIL_SMALL=1
timeout -k 10 200 python3 -u tools/tail_timeline.py run > $OUT/wall.json 2> $OUT/wall.err || { tail -20 $OUT/wall.err; exit 1; }
cat $OUT/wall.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- \
  python3 $R/tools/tail_timeline.py run > $OUT/traced.json 2> $OUT/trace.log || { tail -5 $OUT/trace.log; exit 2; }
T=$(ls $OUT/trace/*kernel_trace.csv $OUT/trace/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 $R/tools/tail_timeline.py show $T > $OUT/timeline.txt || exit 3
rm -f $T
cat $OUT/timeline.txt
