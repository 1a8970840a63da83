#!/bin/bash
# round-2 final pass, part A: every GPU test, then every bench workload (with CPU baselines)
set -o pipefail
TAG=${1:-r02f}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py > $O/bench_vit_c2.json 2> $O/bench_vit_c2.err || exit $?
timeout -k 10 300 python bench.py --workload vit_c4_soap --no-lm > $O/bench_vit_c4_soap.json 2> $O/bench_vit_c4_soap.err || exit $?
timeout -k 10 300 python bench.py --workload vit_c4_shampoo --no-lm > $O/bench_vit_c4_shampoo.json 2> $O/bench_vit_c4_shampoo.err || exit $?
timeout -k 10 400 python bench.py --workload lm124m --steps 10 --warmup 2 > $O/bench_lm124m.json 2> $O/bench_lm124m.err || exit $?
timeout -k 10 400 python bench.py --workload lm420m --steps 3 --warmup 1 > $O/bench_lm420m.json 2> $O/bench_lm420m.err || exit $?
echo benches done
