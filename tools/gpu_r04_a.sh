#!/bin/bash
# round 4: the new parity tests + short-attention phase stamps
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04a
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
PLAINCV_HIP_LIB=$GRAFT_REPO_ROOT/scratch/v/libshtime.so timeout -k 10 120 python tools/sh_phases.py > $O/sh_phases.txt 2>&1 || { tail -20 $O/sh_phases.txt; exit 1; }
grep -v amdgpu.ids $O/sh_phases.txt
timeout -k 10 900 python -u -m pytest "$@" -m gpu -v -s --tb=short --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -15
exit $rc
