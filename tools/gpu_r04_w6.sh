#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04w6
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py -m gpu -q -rA --tb=short --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed" $O/tests.log | cut -c1-200
exit $rc
