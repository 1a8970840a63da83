#!/bin/bash
# round-3 pass A: every GPU test, then the ViT bench lines (C2 default, fp32 C4 SOAP / Shampoo)
set -o pipefail
TAG=${1:-r03a}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python bench.py > $O/bench_vit_c2.json 2> $O/bench_vit_c2.err || exit $?
timeout -k 10 200 python bench.py --workload vit_c4_soap --no-lm > $O/bench_vit_c4_soap.json 2> $O/bench_vit_c4_soap.err || exit $?
timeout -k 10 200 python bench.py --workload vit_c4_shampoo --no-lm > $O/bench_vit_c4_shampoo.json 2> $O/bench_vit_c4_shampoo.err || exit $?
echo benches done
