#!/bin/bash
set -o pipefail
TAG=${1:-r05j}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export PYTHONPATH=$R
cd $R
timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_bench_path_gpu.py tests/test_dp_gpu.py tests/test_golden.py tests/test_kernels_gpu.py > $O/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $O/tests.log | tail -8
grep "BENCHPATH vit_c2 PARAM3" $O/tests.log | sort -k6 -g -r | head -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
db() { ls $1/*.db $1/*/*.db 2>/dev/null | head -1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_f32 -o p -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sub --no-roofline > $O/prof_f32.log 2>&1 || { tail -20 $O/prof_f32.log; exit 1; }
d=$(db $O/prof_f32)
python3 $R/profiles/summarize_rocpd.py "$d" 23 > $O/${TAG}_vit_c2_f32_kernel_stats.txt || exit 1
python3 $R/profiles/step_timeline.py "$d" > $O/${TAG}_vit_c2_f32_step_timeline.txt || exit 1
rm -rf $O/prof_f32
tail -1 $O/${TAG}_vit_c2_f32_step_timeline.txt
head -25 $O/${TAG}_vit_c2_f32_kernel_stats.txt
