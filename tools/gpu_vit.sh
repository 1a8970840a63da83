#!/bin/bash
# ViT pass: GPU tests, default bench (CPU baseline), kernel-trace stats, HBM PMC passes on the LN-bwd GEMM
set -e
TAG=${1:-vit}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py > $O/bench_vit.json 2> $O/bench_vit.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_vit -o p -- python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_vit.log 2>&1
export PYTHONPATH=$R KBENCH_REPS=4 KBENCH_ROUNDS=1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o p -- python $R/tools/kbench.py lnbwd > $O/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o p -- python $R/tools/kbench.py lnbwd > $O/pmc_write.log 2>&1
echo done
