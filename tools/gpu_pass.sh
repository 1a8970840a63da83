#!/bin/bash
# One GPU pass on the box (run through gpurun from the repo root):
#   tools/gpu_pass.sh TAG "PYTEST_ARGS" "BENCH_ARGS"
# PYTEST_ARGS: test selection (e.g. "tests -m gpu", "tests/test_x.py -k y"), "" skips the tests;
# "smoke" as the 4th argument also runs __graft_entry__.smoke(); BENCH_ARGS: bench.py arguments,
# "-" skips the bench.  Every GPU step has its own time limit and a failure ends the pass.
set -o pipefail
TAG=${1:?tag}
TESTS=${2:-}
BENCH=${3:--}
SMOKE=${4:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
export PYTHONPATH=$R
if [ -n "$TESTS" ]; then
  eval "targs=($TESTS)"   # quoted pieces (e.g. -k "a or b") stay one argument
  timeout -k 10 1100 python -u -m pytest "${targs[@]}" -v -s --tb=short --timeout 600 --timeout-method thread \
    > "$O/tests.log" 2>&1
  rc=$?
  grep -E "FAILED|ERROR" "$O/tests.log" | head -20
  tail -1 "$O/tests.log"
  [ $rc -eq 0 ] || exit $rc
fi
if [ "$SMOKE" = "smoke" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
  tail -1 "$O/smoke.log"
fi
if [ "$BENCH" != "-" ]; then
  s0=$(date +%s)
  timeout -k 10 500 python bench.py $BENCH > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
  echo "bench wall $(( $(date +%s) - s0 )) s"
  python tools/bench_summary.py "$O/bench.json"
fi
