#!/bin/bash
# saved GELU derivative: tests, then C2 A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04s
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_vit_parity_gpu.py tests/test_engine_parity_gpu.py -m gpu -x -q --tb=short --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
c2() {   # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-lm --no-f32 > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$tag.json')); print('$tag', d['value'], d['ms_per_step'])"
}
for r in 1 2; do c2 geld_$r X=1 && c2 gel_$r PCV_VIT_GELU_D=0 || exit 1; done
