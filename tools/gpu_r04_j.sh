#!/bin/bash
# round 4: XCD placement defaults (attention heads, embed+LN rows) A/B on C2; LM attention packed-math A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04j
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_vit_parity_gpu.py -m gpu -x -q --tb=short --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
c2() {   # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-lm --no-f32 > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$tag.json')); print('$tag', d['value'], d['ms_per_step'])"
}
lm() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload lm124m --steps 5 --warmup 2 --no-cpu-baseline > $O/lm_$tag.json 2> $O/lm_$tag.err || { tail -20 $O/lm_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/lm_$tag.json')); print('lm124m $tag', d['value'], d['ms_per_step'])"
}
c2 xcd_1 X=1 && c2 xcd_0 PCV_ATTN_XCD=0 && c2 xcd_1b X=1 && c2 xcd_0b PCV_ATTN_XCD=0
lm new X=1 && lm old PLAINCV_HIP_LIB=$GRAFT_REPO_ROOT/tools/bin/v/liblmold.so && lm new2 X=1 && lm old2 PLAINCV_HIP_LIB=$GRAFT_REPO_ROOT/tools/bin/v/liblmold.so
