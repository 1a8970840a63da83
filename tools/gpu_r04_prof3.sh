#!/bin/bash
# final-tree C2 kernel table + step sequence (rocprofv3 kernel trace)
set -o pipefail
TAG=${1:-r04x}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
db() { ls $1/*.db $1/*/*.db 2>/dev/null | head -1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_vit_c2 -o p -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-lm --no-f32 > $O/prof_vit_c2.log 2>&1 || exit $?
d=$(db $O/prof_vit_c2)
python3 $R/profiles/summarize_rocpd.py "$d" 23 > $O/${TAG}_vit_c2_kernel_stats.txt || exit 1
python3 $R/profiles/step_timeline.py "$d" > $O/${TAG}_vit_c2_step_timeline.txt || exit 1
rm -rf $O/prof_vit_c2
tail -1 $O/${TAG}_vit_c2_step_timeline.txt
cd $R
timeout -k 10 400 python bench.py > $O/bench_vit_c2.json 2> $O/bench_vit_c2.err || { tail -20 $O/bench_vit_c2.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_vit_c2.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['vit_c2_f32']['value'], d['lm124m']['value'])"
