#!/bin/bash
# one BOHB refit at 400 / 1e4 observations: wall / native / stream time, and its kernels under rocprof
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/${1:-r04s}
mkdir -p $OUT
for n in 400 10000; do
  timeout -k 10 120 python3 -u tools/refit_host.py $n 2>>$OUT/err.log | tee -a $OUT/host.txt || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $R/tools/refit_host.py 400 > /dev/null 2>> $OUT/err.log || exit 2
T=$(ls $OUT/trace/*kernel_trace.csv $OUT/trace/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 $R/tools/ksteady.py $T --skip 3 > $OUT/steady.txt || exit 3
rm -f $T
head -30 $OUT/steady.txt
