#!/bin/bash
# exact re-score / final variants: wall time per drop-in call at config #2 / #3 (alternated), then two traces
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/${1:-r04k}
mkdir -p $OUT
V=("HBX_LIB_PATH=ab/libhbx_base.so" "HBX_EXACT_FINAL=0 HBX_EXACT32=0" "HBX_EXACT_FINAL=0 HBX_EXACT32=1"
   "HBX_EXACT_FINAL=1 HBX_EXACT32=0 HBX_EXACT_GRID=512" "HBX_EXACT_FINAL=1 HBX_EXACT32=0"
   "HBX_EXACT_FINAL=0 HBX_EXACT32=0 HBX_EXACT_GRID=512")
for i in 1 2; do
  for v in "${V[@]}"; do
    r=$(export $v; timeout -k 10 200 python3 -u tools/tail_timeline.py run 2>> $OUT/wall.err) || { tail -20 $OUT/wall.err; exit 2; }
    echo "$v :: $r" | tee -a $OUT/wall.txt
  done
done
cd /tmp && export TMPDIR=/tmp
for t in "HBX_EXACT_FINAL=0 HBX_EXACT32=0" "HBX_EXACT_FINAL=1 HBX_EXACT32=0 HBX_EXACT_GRID=512"; do
  n=$(echo $t | tr ' =' '__')
  (export $t; timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_$n -o run -- \
    python3 $R/tools/tail_timeline.py run > /dev/null 2> $OUT/trace.log) || { tail -5 $OUT/trace.log; exit 4; }
  T=$(ls $OUT/trace_$n/*kernel_trace.csv $OUT/trace_$n/*/*kernel_trace.csv 2>/dev/null | head -1)
  python3 $R/tools/tail_timeline.py show $T > $OUT/timeline_$n.txt || exit 5
  rm -f $T
  echo "== $t"; cat $OUT/timeline_$n.txt | grep -v "^---" | head -12; grep -A8 "=== config3" $OUT/timeline_$n.txt
done
