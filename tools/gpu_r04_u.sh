#!/bin/bash
# Muon split apply (PCV_MUON_SPLIT_APPLY): overlap tests, then C2 A/B split off / on, alternated
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04u
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
timeout -k 10 400 python -u -m pytest tests/test_vit_parity_gpu.py tests/test_engine_parity_gpu.py -m gpu -x -q --tb=short --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for v in 0 1; do
    PCV_MUON_SPLIT_APPLY=$v timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-lm --no-f32 > $O/s${v}_$r.json 2> $O/s${v}_$r.err || { tail -20 $O/s${v}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/s${v}_$r.json')); print('split=$v', d['value'], d['ms_per_step'])"
  done
done
