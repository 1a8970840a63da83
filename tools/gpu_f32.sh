#!/bin/bash
# fp32 ViT check: its GPU tests, a C4 SOAP bench line and a kernel-trace profile of the same step.
set -o pipefail
T=${1:-f32}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread $R/tests/test_vit_f32_gpu.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 200 python $R/bench.py --workload vit_c4_soap --steps 30 --warmup 10 --no-lm --no-cpu-baseline > $O/c4.json 2> $O/c4.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --workload vit_c4_soap --steps 20 --warmup 5 --no-lm --no-cpu-baseline > $O/p.json 2> $O/p.err || exit $?
echo done
