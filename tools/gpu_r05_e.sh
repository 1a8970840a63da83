#!/bin/bash
# round-5: the whole GPU suite (no -x: every failure listed), then the default bench line
set -o pipefail
TAG=${1:-r05e}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export PYTHONPATH=$R
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $O/tests.log | tail -25
grep -E "BENCHPATH .*loss|C4_SOAP|C4_SHAMPOO|OVERLAP" $O/tests.log | cut -c1-600 | head -12
exit $rc
