#!/bin/bash
# Targeted GPU check (run through gpurun from the repo root): tools/gpu_quick.sh TAG "PYTEST_ARGS" [cmd ...]
# runs the selected tests, then each extra command (a quoted string) under its own time limit.
set -o pipefail
TAG=${1:?tag}; TESTS=${2:-}; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p "$O"; cd "$R" || exit 1
export PYTHONPATH=$R
if [ -n "$TESTS" ]; then
  eval "targs=($TESTS)"
  timeout -k 10 900 python -u -m pytest "${targs[@]}" -v -s --tb=short --timeout 600 --timeout-method thread > "$O/tests.log" 2>&1
  rc=$?; grep -E "FAILED|ERROR" "$O/tests.log" | head -20; tail -1 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
fi
i=0
for c in "$@"; do
  i=$((i + 1))
  timeout -k 10 400 bash -c "$c" > "$O/cmd$i.log" 2>&1 || { echo "cmd$i failed: $c"; tail -20 "$O/cmd$i.log"; exit 1; }
  echo "== cmd$i: $c"; grep -v "amdgpu.ids" "$O/cmd$i.log" | tail -12
done
