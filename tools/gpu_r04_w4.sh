#!/bin/bash
# overlap-vs-in-step diagnostic, then in-step vs in-step (run-to-run noise) on the 16-class model
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out/r04w4
timeout -k 10 120 python -u tools/overlap_diag16b.py 16 > gpurun_out/r04w4/d16.log 2>&1 || { tail -20 gpurun_out/r04w4/d16.log; exit 1; }
DIAG_BOTH_INSTEP=1 timeout -k 10 120 python -u tools/overlap_diag16b.py 16 > gpurun_out/r04w4/d16_instep.log 2>&1 || { tail -20 gpurun_out/r04w4/d16_instep.log; exit 1; }
grep -E "^it|worst grads" gpurun_out/r04w4/d16.log gpurun_out/r04w4/d16_instep.log | sed 's/worst params.*//' | cut -c1-250
