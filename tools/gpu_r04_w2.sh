#!/bin/bash
# overlap test modes (in_block on an aligned model), then the C4 SOAP test three times in one process
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04w2
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
timeout -k 10 300 python -u -m pytest tests/test_vit_parity_gpu.py -k overlap -m gpu -q --tb=short --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python -u - > $O/soap_rep.log 2>&1 <<'PY'
import torch, sys
sys.path.insert(0, ".")
import tests.test_configs_gpu as t
for r in range(3):
    try:
        t.test_c4_fp32_soap_13_steps_two_refreshes(torch.device("cuda"))
        print("rep", r, "PASS", flush=True)
    except AssertionError as e:
        print("rep", r, "FAIL", str(e)[:300], flush=True)
PY
rc=$?
grep -E "C4_SOAP|rep" $O/soap_rep.log | cut -c1-400
exit $rc
