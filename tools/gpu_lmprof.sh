#!/bin/bash
# LM124M bench + kernel-trace profile
set -e
TAG=${1:-x}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python bench.py --workload lm124m --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_lm124m.json 2> $O/bench_lm124m.err
cat $O/bench_lm124m.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_lm124m -o p -- python $R/bench.py --workload lm124m --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_lm124m.log 2>&1
echo done
