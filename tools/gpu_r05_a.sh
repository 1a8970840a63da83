#!/bin/bash
# round-5 baseline: fp32 C2 kernel table + one step's sequence (no live-roofline launches in the
# trace), per-launch times of the fp32 row GEMMs at the exact C2 shapes.
set -o pipefail
TAG=${1:-r05a}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export PYTHONPATH=$R
cd $R
timeout -k 10 300 python tools/f32_dense_times.py > $O/f32_dense_times.txt 2>&1 || { tail -20 $O/f32_dense_times.txt; exit 1; }
cat $O/f32_dense_times.txt
cd /tmp && export TMPDIR=/tmp
db() { ls $1/*.db $1/*/*.db 2>/dev/null | head -1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_f32 -o p -- python3 $R/bench.py --workload vit_c2_f32 --steps 20 --warmup 3 --no-cpu-baseline --no-lm --no-roofline > $O/prof_f32.log 2>&1 || { tail -20 $O/prof_f32.log; exit 1; }
d=$(db $O/prof_f32)
python3 $R/profiles/summarize_rocpd.py "$d" 23 > $O/${TAG}_vit_c2_f32_kernel_stats.txt || exit 1
python3 $R/profiles/step_timeline.py "$d" > $O/${TAG}_vit_c2_f32_step_timeline.txt || exit 1
rm -rf $O/prof_f32
cat $O/${TAG}_vit_c2_f32_step_timeline.txt
head -30 $O/${TAG}_vit_c2_f32_kernel_stats.txt
