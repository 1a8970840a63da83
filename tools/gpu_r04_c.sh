#!/bin/bash
# round 4: row-panel GEMM -- kernel tests, the ViT parity tests, then the C2 step with and without it
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04c
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_rowgemm_gpu.py tests/test_gemm_gpu.py -m gpu -x -v -s --tb=line --timeout 120 --timeout-method thread > $O/tests_rowgemm.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/tests_rowgemm.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_engine_parity_gpu.py tests/test_vit_parity_gpu.py tests/test_golden.py tests/test_kernels_gpu.py -m gpu -x -v -s --tb=line --timeout 120 --timeout-method thread > $O/tests_vit.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/tests_vit.log | tail -8
[ $rc -ne 0 ] && exit $rc
PLAINCV_HIP_LIB=$GRAFT_REPO_ROOT/scratch/v/libshtime.so timeout -k 10 120 python tools/sh_phases.py > $O/sh_phases.txt 2>&1 || { tail -20 $O/sh_phases.txt; exit 1; }
grep -v amdgpu.ids $O/sh_phases.txt
for v in 1 0 1 0; do
  PCV_ROWGEMM=$v timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-lm --no-f32 > $O/bench_$v.json 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$v.json')); print('rowgemm=$v', d['value'], d['ms_per_step'], d['roofline']['launch_us_by_shape'])"
done
