#!/bin/bash
# weight-stationary fp32 row GEMM: correctness, per-launch times at the C2 shapes, the fp32 step
set -o pipefail
TAG=${1:-r05b}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export PYTHONPATH=$R
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_f32_rows_gpu.py > $O/rows_test.log 2>&1 || { tail -30 $O/rows_test.log; exit 1; }
tail -2 $O/rows_test.log
timeout -k 10 300 python tools/f32_dense_times.py > $O/f32_dense_times.txt 2>&1 || { tail -20 $O/f32_dense_times.txt; exit 1; }
cat $O/f32_dense_times.txt
timeout -k 10 300 python bench.py --workload vit_c2_f32 --no-cpu-baseline --no-lm > $O/bench_f32.json 2> $O/bench_f32.err || { tail -20 $O/bench_f32.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_f32.json')); print('vit_c2_f32', d['value'], d['ms_per_step'], d['final_loss'])"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vit_f32_gpu.py tests/test_configs_gpu.py > $O/f32_tests.log 2>&1 || { tail -30 $O/f32_tests.log; exit 1; }
tail -2 $O/f32_tests.log
