#!/bin/bash
# usage: tools/gpu_quick.sh TAG  -- GPU tests, ViT bench, ViT kernel-trace profile
set -e
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --tb=short --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -3 gpurun_out/tests_$TAG.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_vit_$TAG.json 2> gpurun_out/bench_vit_$TAG.err
cat gpurun_out/bench_vit_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_vit_$TAG -o vit -- python $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_vit_$TAG.log 2>&1
echo done
