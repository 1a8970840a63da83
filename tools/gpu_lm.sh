#!/bin/bash
# LM tests + 124M and 420M benches (+ CPU baselines) + kernel traces
set -e
TAG=${1:-lm}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_lm_parity_gpu.py -x -q --tb=short --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python bench.py --workload lm124m --steps 10 --warmup 2 --cpu-seconds 10 > $O/bench_lm124m.json 2> $O/bench_lm124m.err
cat $O/bench_lm124m.json
timeout -k 10 400 python bench.py --workload lm420m --steps 3 --warmup 1 --cpu-seconds 10 > $O/bench_lm420m.json 2> $O/bench_lm420m.err
cat $O/bench_lm420m.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_lm420m -o p -- python $R/bench.py --workload lm420m --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_lm420m.log 2>&1
echo done
