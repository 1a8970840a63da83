#!/bin/bash
# round-3 final pass, part B: kernel-trace profiles of every workload (summarised on the box:
# per-kernel table + one step's kernel sequence for the ViT lines), then the HBM PMC passes of the
# roofline kernels (bf16 ViT: the LN-backward GEMM via kbench; fp32 ViT: the fused attention
# backward), each pass under its own kill timeout.  Databases are removed after summarising
# (gpurun copies back at most 64 MiB).
set -o pipefail
TAG=${1:-r03}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
db() { ls $1/*.db $1/*/*.db 2>/dev/null | head -1; }
summ() {   # name steps [step-timeline]
  local d=$(db $O/prof_$1)
  python3 $R/profiles/summarize_rocpd.py "$d" $2 > $O/${TAG}_$1_kernel_stats.txt || return 1
  if [ -n "$3" ]; then python3 $R/profiles/step_timeline.py "$d" > $O/${TAG}_$1_step_timeline.txt || return 1; fi
  rm -rf $O/prof_$1
}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_vit_c2 -o p -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-lm > $O/prof_vit_c2.log 2>&1 || exit $?
summ vit_c2 23 1 || exit 1
for W in vit_c4_soap vit_c4_shampoo; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$W -o p -- python3 $R/bench.py --workload $W --steps 20 --warmup 3 --no-cpu-baseline --no-lm > $O/prof_$W.log 2>&1 || exit $?
  summ $W 23 1 || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_lm124m -o p -- python3 $R/bench.py --workload lm124m --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_lm124m.log 2>&1 || exit $?
summ lm124m 4 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_lm420m -o p -- python3 $R/bench.py --workload lm420m --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_lm420m.log 2>&1 || exit $?
summ lm420m 3 || exit 1
echo traces done
export PYTHONPATH=$R KBENCH_REPS=4 KBENCH_ROUNDS=1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o p -- python3 $R/tools/kbench.py lnbwd > $O/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o p -- python3 $R/tools/kbench.py lnbwd > $O/pmc_write.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_f32_fetch -o p -- python3 $R/bench.py --workload vit_c4_soap --steps 3 --warmup 1 --no-cpu-baseline --no-lm > $O/pmc_f32_fetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_f32_write -o p -- python3 $R/bench.py --workload vit_c4_soap --steps 3 --warmup 1 --no-cpu-baseline --no-lm > $O/pmc_f32_write.log 2>&1 || exit $?
J=$O/${TAG}_pmc_traffic.json
rm -f $J
(cd $R/profiles && python3 pmc_traffic.py "$(db $O/pmc_fetch)" "$(db $O/pmc_write)" "gemm_bf16_kernel<true, true, 2, 4>" $J \
   && python3 pmc_traffic.py "$(db $O/pmc_f32_fetch)" "$(db $O/pmc_f32_write)" "attn_bwd_f32_kshare_kernel<true>" $J) > $O/${TAG}_pmc_traffic.txt 2>&1 || exit 1
rm -rf $O/pmc_fetch $O/pmc_write $O/pmc_f32_fetch $O/pmc_f32_write
echo done
