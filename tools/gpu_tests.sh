#!/bin/bash
# full GPU test pass into gpurun_out/$1/tests.log
O=gpurun_out/${1:-tests}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --tb=short --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/tests.log | head -20
tail -2 $O/tests.log
exit $rc
