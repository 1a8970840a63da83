#!/bin/bash
# SOAP/Shampoo ViT (BASELINE configs[3] optimizers) bench + kernel trace
set -e
TAG=${1:-c4}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for W in vit_c4_soap vit_c4_shampoo; do
  timeout -k 10 300 python bench.py --workload $W --cpu-seconds 10 > $O/bench_$W.json 2> $O/bench_$W.err
  cat $O/bench_$W.json
done
cd /tmp && export TMPDIR=/tmp
for W in vit_c4_soap vit_c4_shampoo; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$W -o p -- python $R/bench.py --workload $W --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_$W.log 2>&1
done
echo done
