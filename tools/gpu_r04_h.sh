#!/bin/bash
# attention backward A/B: short-path tests, phase stamps of both backward forms, C2 step with each
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04h
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -m gpu -x -q --tb=short --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
PLAINCV_HIP_LIB=$GRAFT_REPO_ROOT/tools/bin/v/libsh.so timeout -k 10 120 python tools/sh_phases.py > $O/sh_phases.txt 2>&1 || { tail -20 $O/sh_phases.txt; exit 1; }
grep -v amdgpu.ids $O/sh_phases.txt
PCV_ATTN_BWD_KEY_OWNED=1 PLAINCV_HIP_LIB=$GRAFT_REPO_ROOT/tools/bin/v/libsh.so timeout -k 10 120 python tools/sh_phases.py > $O/sh_phases_key_owned.txt 2>&1 || { tail -20 $O/sh_phases_key_owned.txt; exit 1; }
grep bwd $O/sh_phases_key_owned.txt
run() {   # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-lm --no-f32 > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$tag.json')); print('$tag', d['value'], d['ms_per_step'])"
}
run base X=1 && run keyowned PCV_ATTN_BWD_KEY_OWNED=1 && run base2 X=1 && run keyowned2 PCV_ATTN_BWD_KEY_OWNED=1
