#!/bin/bash
# panel-form row GEMM: correctness (rows tests + fp32 ViT tests) then per-launch times vs the tiled form
set -o pipefail
TAG=${1:-r05k}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export PYTHONPATH=$R
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_f32_rows_gpu.py > $O/rows.log 2>&1 || { tail -30 $O/rows.log; exit 1; }
tail -2 $O/rows.log
timeout -k 10 300 python -u tools/f32_dense_times.py > $O/f32_dense_times.txt 2>&1 || { tail -20 $O/f32_dense_times.txt; exit 1; }
cat $O/f32_dense_times.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vit_f32_gpu.py tests/test_bench_path_gpu.py -s > $O/f32_tests.log 2>&1
rc=$?
grep -E "passed|failed|^FAILED" $O/f32_tests.log | tail -5
grep "BENCHPATH vit_c2 PARAM3" $O/f32_tests.log | sort -k6 -g -r | head -6
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-sub --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
