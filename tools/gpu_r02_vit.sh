#!/bin/bash
# the three ViT bench lines (C2 default with its attached LM line, fp32 C4 SOAP / Shampoo) + a C4 SOAP kernel trace
set -o pipefail
TAG=${1:-r02j}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py > $O/bench_vit_c2.json 2> $O/bench_vit_c2.err || exit $?
timeout -k 10 300 python bench.py --workload vit_c4_soap --no-lm > $O/bench_vit_c4_soap.json 2> $O/bench_vit_c4_soap.err || exit $?
timeout -k 10 300 python bench.py --workload vit_c4_shampoo --no-lm > $O/bench_vit_c4_shampoo.json 2> $O/bench_vit_c4_shampoo.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_vit_c4_soap -o p -- python3 $R/bench.py --workload vit_c4_soap --steps 20 --warmup 3 --no-cpu-baseline --no-lm > $O/prof_vit_c4_soap.log 2>&1 || exit $?
echo done
