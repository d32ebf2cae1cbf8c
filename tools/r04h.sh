#!/bin/bash
# kernel timelines of the headline step: rescue inside the combine (default) vs the separate rescue pass
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/${1:-r04h}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  HBX_RESCUE_PASS=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_$v -o run -- \
    python3 $R/tools/step_breakdown.py --steps 10 > $OUT/bd_$v.json 2>&1 || exit 1
  T=$(ls $OUT/trace_$v/*kernel_trace.csv $OUT/trace_$v/*/*kernel_trace.csv 2>/dev/null | head -1)
  python3 $R/tools/step_timeline.py $T > $OUT/timeline_$v.txt || exit 2
  rm -f $T
  echo "== HBX_RESCUE_PASS=$v"; tail -17 $OUT/timeline_$v.txt; grep median $OUT/bd_$v.json | cut -c1-400
done
