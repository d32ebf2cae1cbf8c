#!/bin/bash
# The secondary kernels' measurement set on ONE GPU box (run via gpurun), every file from the same session:
#   1. tools/side_kernels.py under rocprofv3 --kernel-trace --stats (durations, no counters),
#   2. four --pmc passes of the same script, one counter group per run (rocprofv3 does not split groups),
#   3. tools/side_roofline.py: per kernel the trace's steady duration, the counters per dispatch and each
#      kernel's roofline fraction on its algorithmic basis.
#   bash tools/profile_side.sh r06/side [WORKLOADS...]   -> gpurun_out/r06/side/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $R/tools/side_kernels.py "$@" > $OUT/side_lines.jsonl 2> $OUT/trace.log || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
           "FETCH_SIZE" "WRITE_SIZE GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set -d $OUT/pmc$i -o run --output-format csv -- \
    python3 $R/tools/side_kernels.py "$@" > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.log; exit 2; }
  echo "pmc pass $i done"
done
cd $R
T=$(ls $OUT/trace/*kernel_trace.csv | head -1)
python3 tools/side_roofline.py $T $OUT > $OUT/side_roofline.txt || exit 3
cp $(ls $OUT/trace/*kernel_stats.csv | head -1) $OUT/kernel_stats.csv
python3 tools/ksteady.py $T --skip 2 > $OUT/kernel_steady.txt || exit 4
rm -rf $OUT/pmc[0-9]/
cat $OUT/side_roofline.txt
echo side profile done
