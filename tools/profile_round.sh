#!/bin/bash
# One round's measurement set on ONE GPU box (run via gpurun), every file from the same session:
#   1. the default bench line (what the driver runs),
#   2. the same bench under rocprofv3 --kernel-trace --stats: its JSON line and the kernel trace come from
#      ONE process, so the line's per-launch HIP-event times and rocprof's durations describe the same
#      launches (tools/ksteady.py reads the trace; tools/trace_vs_line.py checks the two agree),
#   3. PMC passes (traffic, issue, clock) of the scoring step, each pass its own run.
#   bash tools/profile_round.sh r03      -> gpurun_out/r03/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $R/bench.py --no-cpu --profile-tag profiles/$TAG > $OUT/bench_traced.json 2> $OUT/trace.log || { echo "trace failed"; tail -5 $OUT/trace.log; exit 2; }
B="$R/bench.py --steps 5 --warmup 1 --no-cpu --no-config5"
i=0
for set in "FETCH_SIZE" "WRITE_SIZE GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/pmc$i -o run --output-format csv -- python3 $B > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.log; exit 3; }
done
cd $R
W=kde_acquisition_d32_24c8u_obs10000_cand1000000
T=$(ls $OUT/trace/*kernel_trace.csv | head -1)
python3 tools/pmc_summary.py $OUT --kernel kde_logpdf_h --traffic-out $OUT/pmc_traffic.json --workload $W --trace $T > $OUT/pmc_summary.txt || exit 4
python3 tools/ksteady.py $T --skip 3 > $OUT/kernel_steady.txt || exit 5
python3 tools/trace_vs_line.py $T $OUT/bench_traced.json $OUT/bench.json > $OUT/trace_vs_line.txt || exit 6
cp $(ls $OUT/trace/*kernel_stats.csv | head -1) $OUT/kernel_stats.csv
rm -rf $OUT/pmc[0-9]/ $OUT/trace/*kernel_trace.csv
head -8 $OUT/kernel_steady.txt
cat $OUT/trace_vs_line.txt

# package power / clock while the scoring launch runs back to back (is it held at the power limit?)
bash tools/power_trace.sh $OUT/power 8 > $OUT/power.log 2>&1 || { echo "power trace failed"; tail -5 $OUT/power.log; }
grep -i -E "power|sclk|gfx_clk|clock|temp" $OUT/power/samples.txt | head -40
echo profile done
