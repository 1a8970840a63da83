#!/bin/bash
# full measurement pass: tests, benches (ViT w/ CPU baseline, LM), kernel traces, HBM PMC on the roofline kernel
set -e
TAG=${1:-full}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --tb=short --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python bench.py > $O/bench_vit.json 2> $O/bench_vit.err
cat $O/bench_vit.json
timeout -k 10 400 python bench.py --workload lm124m --steps 5 --warmup 2 > $O/bench_lm.json 2> $O/bench_lm.err
cat $O/bench_lm.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_vit -o vit -- python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_vit.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_lm -o lm -- python $R/bench.py --workload lm124m --steps 3 --warmup 1 > $O/prof_lm.log 2>&1
export PYTHONPATH=$R KBENCH_REPS=4 KBENCH_ROUNDS=1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o p -- python $R/tools/kbench.py lnbwd > $O/pmc_fetch.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o p -- python $R/tools/kbench.py lnbwd > $O/pmc_write.log 2>&1
echo done
