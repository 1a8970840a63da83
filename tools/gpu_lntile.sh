#!/bin/bash
# pcv_gemm_ln tile-height experiment: 64-row (default) vs 32-row tiles, per launch and in the C2 step
set -o pipefail
TAG=${1:-lntile}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 180 python tools/ln_tail.py > $O/tail64.txt 2>&1 || { tail -20 $O/tail64.txt; exit 1; }
cat $O/tail64.txt
PCV_LN_TILE=32 timeout -k 10 180 python tools/ln_tail.py > $O/tail32.txt 2>&1 || { tail -20 $O/tail32.txt; exit 1; }
cat $O/tail32.txt
for t in 64 32 64 32; do
  PCV_LN_TILE=$t timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-lm > $O/bench_$t.json 2> $O/bench_$t.err || { tail -20 $O/bench_$t.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$t.json')); print('tile $t', d['value'], d['ms_per_step'])"
done
