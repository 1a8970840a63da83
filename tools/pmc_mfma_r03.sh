#!/bin/bash
# MFMA utilisation per kernel for every bench workload (round 3): two rocprofv3 --pmc passes per
# workload (busy cycles / MFMA instruction counts), each under its own kill timeout, summarised
# on the box by profiles/mfma_util.py into $TAG/<workload>_mfma_util.txt (databases removed).
TAG=${1:-r03_mfma}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run_pass() {   # name workload-args counters...
  local name=$1; shift
  local wl=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $O/$name -o p -- python3 $R/bench.py $wl --no-cpu-baseline --no-lm > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
for spec in "vit_c2|--steps 10 --warmup 2" "vit_c4_soap|--workload vit_c4_soap --steps 10 --warmup 2" \
            "vit_c4_shampoo|--workload vit_c4_shampoo --steps 10 --warmup 2" \
            "lm124m|--workload lm124m --steps 1 --warmup 1 --lm-accum 2"; do
  name=${spec%%|*}; wl=${spec#*|}
  run_pass ${name}_busy "$wl" SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
  run_pass ${name}_insts "$wl" SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_WAVE_CYCLES
  B=$(ls $O/${name}_busy/*.db $O/${name}_busy/*/*.db 2>/dev/null | head -1)
  I=$(ls $O/${name}_insts/*.db $O/${name}_insts/*/*.db 2>/dev/null | head -1)
  (cd $R/profiles && python3 mfma_util.py "$B" "$I" $O/${name}_mfma_util.txt --top 30) > /dev/null 2>&1
  rm -rf $O/${name}_busy $O/${name}_insts
done
ls $O
