#!/bin/bash
# full measurement pass for a round: GPU tests; every bench workload (with CPU baselines);
# kernel-trace stats of each; HBM PMC passes on the ViT roofline kernel
set -e
TAG=${1:-round}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py > $O/bench_vit.json 2> $O/bench_vit.err
timeout -k 10 300 python bench.py --workload vit_c4_soap --cpu-seconds 10 > $O/bench_vit_c4_soap.json 2> $O/bench_vit_c4_soap.err
timeout -k 10 300 python bench.py --workload vit_c4_shampoo --cpu-seconds 10 > $O/bench_vit_c4_shampoo.json 2> $O/bench_vit_c4_shampoo.err
timeout -k 10 400 python bench.py --workload lm124m --steps 10 --warmup 2 --cpu-seconds 10 > $O/bench_lm124m.json 2> $O/bench_lm124m.err
timeout -k 10 400 python bench.py --workload lm420m --steps 3 --warmup 1 --cpu-seconds 10 > $O/bench_lm420m.json 2> $O/bench_lm420m.err
echo benches done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_vit -o p -- python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_vit.log 2>&1
for W in vit_c4_soap vit_c4_shampoo; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$W -o p -- python $R/bench.py --workload $W --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_$W.log 2>&1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_lm124m -o p -- python $R/bench.py --workload lm124m --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_lm124m.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_lm420m -o p -- python $R/bench.py --workload lm420m --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_lm420m.log 2>&1
echo traces done
export PYTHONPATH=$R KBENCH_REPS=4 KBENCH_ROUNDS=1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o p -- python $R/tools/kbench.py lnbwd > $O/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o p -- python $R/tools/kbench.py lnbwd > $O/pmc_write.log 2>&1
echo done
