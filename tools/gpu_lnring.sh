#!/bin/bash
# pcv_gemm_ln ring depth: the default library (2 stages) vs variants built with
# -DPCV_GEMM_STAGES_LN=3/4 (scratch/v/libS*.so, selected by PLAINCV_HIP_LIB): per launch cold/warm, C2 step
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/lnring
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
for v in S2 S3 S4; do
  if [ $v = S2 ]; then unset PLAINCV_HIP_LIB; else export PLAINCV_HIP_LIB=$GRAFT_REPO_ROOT/scratch/v/lib$v.so; fi
  timeout -k 10 200 python tools/ln_tail.py > $O/tail_$v.txt 2>&1 || { tail -20 $O/tail_$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/tail_$v.txt
done
for v in S2 S3 S4 S2 S3 S4; do
  if [ $v = S2 ]; then unset PLAINCV_HIP_LIB; else export PLAINCV_HIP_LIB=$GRAFT_REPO_ROOT/scratch/v/lib$v.so; fi
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-lm > $O/bench_$v.json 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$v.json')); print('$v', d['value'], d['ms_per_step'])"
done
