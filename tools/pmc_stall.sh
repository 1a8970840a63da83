#!/bin/bash
# Issue / stall counters per kernel (one rocprofv3 --pmc pass per group, each under its own kill
# timeout): tools/pmc_stall.sh TAG "bench args" [python script, default bench.py]
TAG=${1:-r03_stall}
WL=${2:-"--steps 10 --warmup 2"}
PROG=${3:-bench.py}
EXTRA=""
if [ "$PROG" = "bench.py" ]; then EXTRA="--no-cpu-baseline --no-lm --no-f32"; fi
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
run_pass() {   # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $O/$name -o p -- python3 $R/$PROG $WL $EXTRA > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
run_pass waits SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES
run_pass insts SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM
# summarise on the box and drop the databases (gpurun copies back at most 64 MiB)
DB1=$(ls $O/waits/*.db $O/waits/*/*.db 2>/dev/null | head -1)
DB2=$(ls $O/insts/*.db $O/insts/*/*.db 2>/dev/null | head -1)
(cd $R/profiles && python3 pmc_stall.py "$DB1" "$DB2" --top 30) > $O/summary.txt 2>&1
du -sh $O/waits $O/insts >> $O/summary.txt
rm -rf $O/waits $O/insts
