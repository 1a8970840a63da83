#!/bin/bash
# XCD order for patchify / embed backward: tests, C2 (compare with the r04y line on another box: use the old tree too)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04t
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_vit_parity_gpu.py tests/test_golden.py tests/test_engine_parity_gpu.py -m gpu -x -q --tb=short --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  (cd $R/tools/bin/oldtree && PYTHONPATH=$R/tools/bin/oldtree timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-lm --no-f32 > $O/old_$r.json 2> $O/old_$r.err) || { tail -20 $O/old_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/old_$r.json')); print('old', d['value'], d['ms_per_step'])"
  (cd $R && timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-lm --no-f32 > $O/new_$r.json 2> $O/new_$r.err) || { tail -20 $O/new_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/new_$r.json')); print('new', d['value'], d['ms_per_step'])"
done
