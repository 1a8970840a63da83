#!/bin/bash
# fp32 ViT model-level checks (oracle parity, bench path, configs, DP) + headline bench + step timeline
set -o pipefail
TAG=${1:-r05q}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export PYTHONPATH=$R
cd $R
timeout -k 10 900 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gemm_f32_rows_gpu.py tests/test_vit_f32_gpu.py tests/test_bench_path_gpu.py tests/test_configs_gpu.py tests/test_golden.py tests/test_dp_gpu.py tests/test_engine_parity_gpu.py > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|^FAILED|^ERROR" $O/tests.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-sub --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o p -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sub --no-roofline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
d=$(ls $O/prof/*.db $O/prof/*/*.db 2>/dev/null | head -1)
python3 $R/profiles/summarize_rocpd.py "$d" 23 > $O/${TAG}_vit_c2_f32_kernel_stats.txt || exit 1
python3 $R/profiles/step_timeline.py "$d" > $O/${TAG}_vit_c2_f32_step_timeline.txt || exit 1
rm -rf $O/prof
tail -1 $O/${TAG}_vit_c2_f32_step_timeline.txt
