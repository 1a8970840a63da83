#!/bin/bash
# round-3 closing pass: kernel-trace profile of the ViT C2 step (per-kernel table + one step's
# kernel sequence), then the fp32 C4 bench lines (SOAP, Shampoo) on the same tree.
set -o pipefail
TAG=${1:-r03h}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
db() { ls $1/*.db $1/*/*.db 2>/dev/null | head -1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_vit_c2 -o p -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-lm > $O/prof_vit_c2.log 2>&1 || exit $?
d=$(db $O/prof_vit_c2)
python3 $R/profiles/summarize_rocpd.py "$d" 23 > $O/${TAG}_vit_c2_kernel_stats.txt || exit 1
python3 $R/profiles/step_timeline.py "$d" > $O/${TAG}_vit_c2_step_timeline.txt || exit 1
rm -rf $O/prof_vit_c2
tail -3 $O/${TAG}_vit_c2_step_timeline.txt
cd $R
for W in vit_c4_soap vit_c4_shampoo; do
  timeout -k 10 300 python bench.py --workload $W --no-lm > $O/bench_$W.json 2> $O/bench_$W.err || exit $?
  python -c "import json; d=json.load(open('$O/bench_$W.json')); print('$W', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
