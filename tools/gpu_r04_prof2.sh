#!/bin/bash
# round-4 profiles: C2 kernel table + step sequence (rocprofv3 kernel trace), HBM PMC traffic of the
# roofline kernels, MFMA utilisation per workload, the fp32 C4 bench lines.
set -o pipefail
TAG=${1:-r04z}
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
bash $R/tools/pmc_traffic_r03.sh ${TAG}_pmc || exit $?
cat $R/gpurun_out/${TAG}_pmc/${TAG}_pmc_traffic.txt
bash $R/tools/pmc_mfma_r03.sh ${TAG}_mfma || exit $?
cd $R
for W in vit_c4_soap vit_c4_shampoo; do
  timeout -k 10 300 python bench.py --workload $W --no-lm > $O/bench_$W.json 2> $O/bench_$W.err || exit $?
  python -c "import json; d=json.load(open('$O/bench_$W.json')); print('$W', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
