#!/bin/bash
# usage: tools/prof_lm.sh TAG -- kernel-trace profile of the 124M LM bench step
set -e
TAG=${1:-x}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_lm_$TAG -o lm -- python $R/bench.py --workload lm124m --steps 3 --warmup 1 > $R/gpurun_out/prof_lm_$TAG.log 2>&1
echo done
