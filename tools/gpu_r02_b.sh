#!/bin/bash
# round-2 final pass, part B: kernel-trace profiles of every workload, HBM PMC passes on the
# roofline kernels (bf16 ViT: LN-backward GEMM via kbench; fp32 ViT: the fused attention backward)
set -o pipefail
TAG=${1:-r02f}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_vit_c2 -o p -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-lm > $O/prof_vit_c2.log 2>&1 || exit $?
for W in vit_c4_soap vit_c4_shampoo; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$W -o p -- python3 $R/bench.py --workload $W --steps 20 --warmup 3 --no-cpu-baseline --no-lm > $O/prof_$W.log 2>&1 || exit $?
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_lm124m -o p -- python3 $R/bench.py --workload lm124m --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_lm124m.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_lm420m -o p -- python3 $R/bench.py --workload lm420m --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_lm420m.log 2>&1 || exit $?
echo traces done
export PYTHONPATH=$R KBENCH_REPS=4 KBENCH_ROUNDS=1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o p -- python3 $R/tools/kbench.py lnbwd > $O/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o p -- python3 $R/tools/kbench.py lnbwd > $O/pmc_write.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_f32_fetch -o p -- python3 $R/bench.py --workload vit_c4_soap --steps 3 --warmup 1 --no-cpu-baseline --no-lm > $O/pmc_f32_fetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_f32_write -o p -- python3 $R/bench.py --workload vit_c4_soap --steps 3 --warmup 1 --no-cpu-baseline --no-lm > $O/pmc_f32_write.log 2>&1 || exit $?
echo done
