#!/bin/bash
# staggered mixed-role short attention backward: tests, phases, C2 A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04r
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -m gpu -x -q --tb=short --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
PLAINCV_HIP_LIB=$GRAFT_REPO_ROOT/tools/bin/v/libsh.so timeout -k 10 120 python tools/sh_phases.py > $O/sh_phases.txt 2>&1 || { tail -20 $O/sh_phases.txt; exit 1; }
grep "bwdR" $O/sh_phases.txt
PCV_ATTN_BWD_MIX=1 PLAINCV_HIP_LIB=$GRAFT_REPO_ROOT/tools/bin/v/libsh.so timeout -k 10 120 python tools/sh_phases.py > $O/sh_phases_mix.txt 2>&1 || { tail -20 $O/sh_phases_mix.txt; exit 1; }
grep "bwdR" $O/sh_phases_mix.txt
c2() {   # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-lm --no-f32 > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$tag.json')); print('$tag', d['value'], d['ms_per_step'])"
}
for r in 1 2; do c2 base_$r X=1 && c2 mix_$r PCV_ATTN_BWD_MIX=1 || exit 1; done
