#!/bin/bash
# One GPU-box session of this round's work (run through gpurun), every step under its own time limit,
# chained so that the first failure ends the session:
#   bash tools/gpu_session.sh TAG tests [PYTEST_ARGS...]   -> the -m gpu suite (or a selection)
#   bash tools/gpu_session.sh TAG bench [BENCH_ARGS...]    -> one bench.py line
#   bash tools/gpu_session.sh TAG both                     -> the suite, then the default bench line
#   bash tools/gpu_session.sh TAG py SCRIPT [ARGS...]      -> a tools/ measurement script
#   bash tools/gpu_session.sh TAG prof SCRIPT [ARGS...]    -> the same under rocprofv3 --kernel-trace --stats
# Output under gpurun_out/TAG/ (merged back by gpurun); copy what is judged into profiles/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
MODE=$2
shift 2
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
run_tests() {
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rfE --maxfail=10 --timeout 300 --timeout-method thread "$@" \
    > $OUT/pytest.log 2>&1
  local rc=$?
  tail -30 $OUT/pytest.log
  return $rc
}
run_bench() {
  timeout -k 10 900 python -u bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
  local rc=$?
  tail -5 $OUT/bench.err
  cat $OUT/bench.json
  return $rc
}
case $MODE in
  tests) run_tests "$@" ;;
  bench) run_bench "$@" ;;
  both) run_tests && run_bench ;;
  py) S=$1; shift; timeout -k 10 900 python -u $S "$@" > $OUT/$(basename $S .py).txt 2>&1; rc=$?; tail -40 $OUT/$(basename $S .py).txt; exit $rc ;;
  prof) S=$1; shift; cd /tmp && export TMPDIR=/tmp && cd $R
    timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 -u $S "$@" \
      > $OUT/$(basename $S .py)_prof.txt 2>&1; rc=$?; tail -20 $OUT/$(basename $S .py)_prof.txt; exit $rc ;;
  *) echo "unknown mode $MODE"; exit 2 ;;
esac
