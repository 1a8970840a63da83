#!/bin/bash
set -o pipefail
TAG=${1:-r05h}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export PYTHONPATH=$R
cd $R
timeout -k 10 300 python tools/overlap_diag5.py > $O/overlap_diag.txt 2>&1; cut -c1-400 $O/overlap_diag.txt
timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_vit_parity_gpu.py tests/test_bench_path_gpu.py tests/test_precond_gpu.py tests/test_vit_f32_gpu.py tests/test_configs_gpu.py tests/test_optim_parity_gpu.py tests/test_dp_gpu.py tests/test_golden.py > $O/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $O/tests.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/f32_dense_times.py > $O/f32_dense_times.txt 2>&1 || { tail -20 $O/f32_dense_times.txt; exit 1; }
tail -3 $O/f32_dense_times.txt
timeout -k 10 300 python bench.py --no-sub --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('headline', d['value'], d['ms_per_step'], d['roofline']['frac'])"
