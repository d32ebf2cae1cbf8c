#!/bin/bash
# Kernel timelines of the headline step under rocprofv3 for the in-tree build and libhbx variants
# (ab/libhbx_<name>.so), one box:  bash tools/timeline_ab.sh <outdir> <name>...   (via gpurun)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in base "$@"; do
  lib=""
  [ "$v" != base ] && lib=$R/ab/libhbx_$v.so
  HBX_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_$v -o run -- \
    python3 $R/tools/step_breakdown.py --steps 10 > $OUT/bd_$v.json 2>&1 || exit 1
  T=$(ls $OUT/trace_$v/*kernel_trace.csv $OUT/trace_$v/*/*kernel_trace.csv 2>/dev/null | head -1)
  python3 $R/tools/step_timeline.py $T > $OUT/timeline_$v.txt || exit 2
  rm -f $T
  echo "== $v"; tail -9 $OUT/timeline_$v.txt
done
