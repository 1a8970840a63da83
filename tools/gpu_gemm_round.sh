#!/bin/bash
# GPU tests + GEMM shape sweep + ViT / LM124M benches (one gpurun call)
set -e
TAG=${1:-x}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
PYTHONPATH=. timeout -k 10 300 python tools/gemm_bench.py "" --ab > $O/gemm.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_vit.json 2> $O/bench_vit.err
cat $O/bench_vit.json
timeout -k 10 400 python bench.py --workload lm124m --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_lm124m.json 2> $O/bench_lm124m.err
cat $O/bench_lm124m.json
