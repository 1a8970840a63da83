#!/bin/bash
# round 4: env-knob A/B on C2 after the XCD placement (LN tile rows, grouped-wgrad block target)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04l
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
c2() {   # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-lm --no-f32 > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$tag.json')); print('$tag', d['value'], d['ms_per_step'])"
}
for r in 1 2; do
  c2 base_$r X=1 && c2 ln32_$r PCV_LN_TILE=32 && c2 wg1024_$r PCV_WGRAD_BLOCKS=1024 && c2 wg4096_$r PCV_WGRAD_BLOCKS=4096 || exit 1
done
