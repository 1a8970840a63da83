#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04w3
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
timeout -k 10 300 python -u -m pytest tests/test_vit_parity_gpu.py tests/test_optim_parity_gpu.py -k "overlap" -m gpu -q -rA --runxfail --tb=short --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "^E  |PASSED|FAILED|passed|failed" $O/tests.log | cut -c1-200
[ $rc -gt 1 ] && exit $rc
exit 0
