set -o pipefail
mkdir -p gpurun_out/r01h
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r01h/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r01h/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r01h/pytest_gpu.log
timeout -k 10 200 python -u bench.py --candidates 100000 --obs 1000 --dc 8 --du 0 --no-cpu --no-config5 > gpurun_out/r01h/bench_c2.json 2> gpurun_out/r01h/err.log || exit 2
HBX_HMODE=0 timeout -k 10 200 python -u bench.py --candidates 100000 --obs 1000 --dc 8 --du 0 --no-cpu --no-config5 > gpurun_out/r01h/bench_c2_f32.json 2>> gpurun_out/r01h/err.log || exit 3
