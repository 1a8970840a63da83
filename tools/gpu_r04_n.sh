#!/bin/bash
# round 4: negated row constants in the short attention backward -- tests, phases, C2
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04n
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_vit_parity_gpu.py tests/test_golden.py -m gpu -x -q --tb=short --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
PLAINCV_HIP_LIB=$GRAFT_REPO_ROOT/tools/bin/v/libsh.so timeout -k 10 120 python tools/sh_phases.py > $O/sh_phases.txt 2>&1 || { tail -20 $O/sh_phases.txt; exit 1; }
grep bwd $O/sh_phases.txt
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-lm --no-f32 > $O/bench_$r.json 2> $O/bench_$r.err || { tail -20 $O/bench_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$r.json')); print('c2', d['value'], d['ms_per_step'])"
done
