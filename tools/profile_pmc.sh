#!/bin/bash
# PMC passes (one rocprofv3 run per pass: counters are not split over passes) on the bench workload.
# Run on the GPU box via gpurun:  bash tools/profile_pmc.sh <outname>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MFMA SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-config5 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
cd $R
python3 tools/pmc_summary.py $OUT --traffic-out $OUT/pmc_traffic.json --workload kde_acquisition_d32_24c8u_obs10000_cand1000000 > $OUT/pmc_summary.txt || exit 1
rm -rf $OUT/p1 $OUT/p2 $OUT/p3 $OUT/p4  # raw per-dispatch CSVs: too large to copy back
echo pmc done
