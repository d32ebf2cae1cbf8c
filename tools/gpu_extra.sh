#!/bin/bash
# After tools/gpu_check.sh: config #2 bench and a 2-rank rehearsal of the multi-process path on one GPU
# (gloo, ranks sharing the card).  Run via gpurun.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-extra}
mkdir -p $OUT
cd $R
timeout -k 10 200 python -u bench.py --candidates 100000 --obs 1000 --dc 8 --du 0 --no-cpu --no-config5 > $OUT/bench_c2.json 2> $OUT/err.log || { echo c2 failed; tail $OUT/err.log; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 2 --backend gloo --share-gpu --no-cpu --no-config5 > $OUT/bench_n2_gloo.json 2>> $OUT/err.log || { echo n2 failed; tail $OUT/err.log; exit 2; }
cat $OUT/bench_n2_gloo.json
