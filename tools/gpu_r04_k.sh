#!/bin/bash
# round 4: weight-gradient split onto a side stream -- parity test, then C2 A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04k
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_vit_parity_gpu.py -k "wgrad_split or overlap" -m gpu -x -q -s --tb=short --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "WGRAD_SPLIT|OVERLAP|passed|failed" $O/tests.log | tail -5
[ $rc -ne 0 ] && exit $rc
c2() {   # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-lm --no-f32 > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$tag.json')); print('$tag', d['value'], d['ms_per_step'])"
}
c2 base X=1 && c2 split PCV_WGRAD_SPLIT=1 && c2 base2 X=1 && c2 split2 PCV_WGRAD_SPLIT=1
