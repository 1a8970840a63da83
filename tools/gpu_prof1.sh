#!/bin/bash
# one workload's bench line + kernel-trace profile: gpu_prof1.sh TAG WORKLOAD [extra bench args]
set -o pipefail
T=$1; W=$2; shift 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
timeout -k 10 200 python $R/bench.py --workload $W --steps 30 --warmup 10 --no-lm --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --workload $W --steps 20 --warmup 5 --no-lm --no-cpu-baseline "$@" > $O/p.json 2> $O/p.err || exit $?
echo done
