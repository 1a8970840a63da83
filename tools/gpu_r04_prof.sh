#!/bin/bash
# round 4 profile pass: default bench line (headline + fp32 sub-line, no LM), the C2 kernel table and
# one step's kernel sequence, per-kernel stall counters, and the lm_head vs hipBLASLt comparison.
set -o pipefail
TAG=${1:-r04b}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export PYTHONPATH=$R
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-lm > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c2.json')); f=d['vit_c2_f32']; print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['launch_us_by_shape'], '| f32', f['value'], f['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
db() { ls $1/*.db $1/*/*.db 2>/dev/null | head -1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_vit_c2 -o p -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-lm --no-f32 > $O/prof_vit_c2.log 2>&1 || exit $?
d=$(db $O/prof_vit_c2)
python3 $R/profiles/summarize_rocpd.py "$d" 23 > $O/${TAG}_vit_c2_kernel_stats.txt || exit 1
python3 $R/profiles/step_timeline.py "$d" > $O/${TAG}_vit_c2_step_timeline.txt || exit 1
rm -rf $O/prof_vit_c2
tail -1 $O/${TAG}_vit_c2_step_timeline.txt
bash $R/tools/pmc_stall.sh ${TAG}_stall "--steps 10 --warmup 2" || exit $?
head -40 $R/gpurun_out/${TAG}_stall/summary.txt
cd $R
timeout -k 10 200 python tools/lmhead_vs_blaslt.py > $O/lmhead_vs_blaslt.txt 2>&1 || { tail -5 $O/lmhead_vs_blaslt.txt; exit 1; }
grep -v amdgpu.ids $O/lmhead_vs_blaslt.txt
