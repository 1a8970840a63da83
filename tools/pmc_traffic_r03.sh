#!/bin/bash
# HBM PMC passes of the two roofline kernels (bf16 ViT: the LN-backward GEMM via kbench; fp32 ViT:
# the fused attention backward in the C4 SOAP step), each pass under its own kill timeout, summed
# into $TAG/${TAG}_pmc_traffic.json by profiles/pmc_traffic.py (databases removed).
set -o pipefail
TAG=${1:-r03_pmc}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
db() { ls $1/*.db $1/*/*.db 2>/dev/null | head -1; }
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
