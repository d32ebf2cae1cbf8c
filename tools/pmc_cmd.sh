#!/bin/bash
# PMC passes (one rocprofv3 run per pass) over an arbitrary python script; summary per kernel.
#   bash tools/pmc_cmd.sh <outname> <script.py> [args...]     (run on the GPU box via gpurun)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
NAME=$1; shift
OUT=$R/gpurun_out/$NAME
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
# PMC_SETS: passes separated by ';' (default: the four below)
SETS=${PMC_SETS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU;SQ_INSTS_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT;FETCH_SIZE;WRITE_SIZE"}
IFS=';' read -ra PASSES <<< "$SETS"
for set in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 "$R/$1" "${@:2}" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
cd $R
python3 tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt || exit 1
rm -rf $OUT/p[0-9]*/
cat $OUT/pmc_summary.txt | head -40
