#!/bin/bash
set -o pipefail
TAG=${1:-r05n}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export PYTHONPATH=$R
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_f32_rows_gpu.py > $O/rows.log 2>&1 || { tail -30 $O/rows.log; exit 1; }
tail -1 $O/rows.log
timeout -k 10 300 python -u tools/panel_probe.py > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
cat $O/probe.txt
timeout -k 10 300 python -u tools/panel_stamps.py > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
grep -E "==|prologue|it0|it1 |end |tail WG" $O/stamps.txt
