#!/bin/bash
# Package power, engine clock and temperature sampled every ~0.25 s while back-to-back config #3
# acquisitions run (tools/power_probe.py), then a few idle samples: is the scoring kernel held at the
# package power limit?      bash tools/power_trace.sh <out_dir> [seconds]
set -o pipefail
O=${1:-gpurun_out/power}
SEC=${2:-8}
mkdir -p $O
timeout 10 amd-smi static -l -g 0 > $O/limits.txt 2>&1 || true   # the power cap
timeout -k 10 120 python -u tools/power_probe.py $SEC > $O/probe.log 2>&1 &
P=$!
sleep 4   # the probe's fit and first launches
end=$((SECONDS + SEC - 1))
while [ $SECONDS -lt $end ] && kill -0 $P 2>/dev/null; do
  echo "--- busy $(date +%s.%N)" >> $O/samples.txt
  timeout 5 amd-smi metric -p -c -t -g 0 >> $O/samples.txt 2>&1 || timeout 5 rocm-smi --showpower --showclocks --showtemp >> $O/samples.txt 2>&1
  sleep 0.25
done
wait $P || { echo "probe failed"; cat $O/probe.log; exit 1; }
for i in 1 2 3; do
  echo "--- idle $(date +%s.%N)" >> $O/samples.txt
  timeout 5 amd-smi metric -p -c -t -g 0 >> $O/samples.txt 2>&1 || timeout 5 rocm-smi --showpower --showclocks --showtemp >> $O/samples.txt 2>&1
  sleep 0.5
done
cat $O/probe.log
echo power trace done
