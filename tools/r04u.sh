#!/bin/bash
# kernel timelines of config #2 / #3 acquisitions: the rescue in the combine kernel against its own launch
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/${1:-r04u}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  HBX_COMBINE_RESCUE=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace$v -o run -- \
    python3 $R/tools/tail_timeline.py run > $OUT/traced$v.json 2> $OUT/trace$v.log || { tail -5 $OUT/trace$v.log; exit 2; }
  T=$(ls $OUT/trace$v/*kernel_trace.csv $OUT/trace$v/*/*kernel_trace.csv 2>/dev/null | head -1)
  python3 $R/tools/tail_timeline.py show $T > $OUT/timeline$v.txt || exit 3
  rm -f $T
done
grep -A9 "=== config3" $OUT/timeline1.txt | head -10
grep -A9 "=== config3" $OUT/timeline0.txt | head -10
