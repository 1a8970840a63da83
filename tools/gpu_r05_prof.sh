#!/bin/bash
# round-5 profiles of the fp32 C2 step (the default bench workload): HBM PMC passes (FETCH_SIZE,
# WRITE_SIZE) summed per kernel into ${TAG}_pmc_traffic.json, MFMA-busy passes into
# ${TAG}_vit_c2_f32_mfma_util.txt, then the kernel table and one step's kernel sequence.  Every pass
# under its own kill timeout; databases removed after summarising.
set -o pipefail
TAG=${1:-r05z}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
db() { ls $1/*.db $1/*/*.db 2>/dev/null | head -1; }
WL="--steps 3 --warmup 1 --no-sub --no-cpu-baseline --no-roofline"
pass() {   # name counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" -d $O/$name -o p -- python3 $R/bench.py $WL > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
pass pmc_fetch FETCH_SIZE
pass pmc_write WRITE_SIZE
J=$O/${TAG}_pmc_traffic.json
rm -f $J
for k in "gemm_f32_panel_kernel<false, 1, 128, 64>" "gemm_f32_panel_kernel<false, 21, 128, 64>" \
         "gemm_f32_rows_kernel<false, true, 128, 32, true, 512>" "attn_bwd_f32_kshare_kernel<true>" \
         "attn_fwd_f32_kernel<true>" "gemm_f32_wgrad_kernel<128>"; do
  echo "== $k"
  (cd $R/profiles && python3 pmc_traffic.py "$(db $O/pmc_fetch)" "$(db $O/pmc_write)" "$k" $J) || exit 1
done > $O/${TAG}_pmc_traffic.txt
rm -rf $O/pmc_fetch $O/pmc_write
pass busy SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
pass insts SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_WAVE_CYCLES
python3 $R/profiles/mfma_util.py "$(db $O/busy)" "$(db $O/insts)" $O/${TAG}_vit_c2_f32_mfma_util.txt --top 30 > /dev/null || exit 1
rm -rf $O/busy $O/insts
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o p -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sub --no-roofline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
d=$(db $O/prof)
python3 $R/profiles/summarize_rocpd.py "$d" 30 > $O/${TAG}_vit_c2_f32_kernel_stats.txt || exit 1
python3 $R/profiles/step_timeline.py "$d" > $O/${TAG}_vit_c2_f32_step_timeline.txt || exit 1
rm -rf $O/prof
tail -1 $O/${TAG}_vit_c2_f32_step_timeline.txt
cat $O/${TAG}_pmc_traffic.txt
