#!/bin/bash
# MFMA-utilisation counters (SQ_VALU_MFMA_BUSY_CYCLES, MFMA instruction counts) for the ViT C2 step
# and the 124M LM step, one rocprofv3 --pmc pass per counter group, each under its own kill timeout.
# A pass that fails with an ordinary error (e.g. a counter this ROCm does not expose) is skipped;
# a pass killed by its timeout or by a signal ends the script.
TAG=${1:-r02_mfma}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
run_pass() {   # name workload-args counters...
  local name=$1; shift
  local wl=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $O/$name -o p -- python3 $R/bench.py $wl --no-cpu-baseline --no-lm > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
VIT="--steps 10 --warmup 2"
LM="--workload lm124m --steps 1 --warmup 1 --lm-accum 2"
run_pass vit_busy "$VIT" SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
run_pass vit_insts "$VIT" SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_WAVE_CYCLES
run_pass lm_busy "$LM" SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
run_pass lm_insts "$LM" SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_WAVE_CYCLES
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace_vit -o p -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-lm > $O/trace_vit.log 2>&1
echo "trace rc=$?"
