#!/bin/bash
# PMC passes over tools/f32gemm_bench.py case $1 (one rocprofv3 --pmc pass per counter group).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_gemm_$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_F32 SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/a -o p -- python3 $R/tools/f32gemm_bench.py $1 > $O/a.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_WAVES SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT -d $O/b -o p -- python3 $R/tools/f32gemm_bench.py $1 > $O/b.log 2>&1 || exit $?
echo done
