#!/bin/bash
# timing experiment: how much of the C2 step is the dropout hash (variant lib with a trivial hash)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04q
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
c2() {   # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-lm --no-f32 > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$tag.json')); print('$tag', d['value'], d['ms_per_step'])"
}
for r in 1 2; do c2 base_$r X=1 && c2 cheap_$r PLAINCV_HIP_LIB=$GRAFT_REPO_ROOT/tools/bin/v/libcheaphash.so || exit 1; done
