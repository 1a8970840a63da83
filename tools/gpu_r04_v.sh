#!/bin/bash
# Muon overlapped NS phase with the update applied in the NS workgroup (PCV_MUON_OVERLAP_IN_BLOCK):
# tests, C2 A/B alternated, then the step timeline of the default
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04v
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
timeout -k 10 500 python -u -m pytest tests/test_vit_parity_gpu.py tests/test_engine_parity_gpu.py tests/test_golden.py tests/test_optim_parity_gpu.py -m gpu -x -q --tb=short --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for v in 0 1; do
    PCV_MUON_OVERLAP_IN_BLOCK=$v timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-lm --no-f32 > $O/b${v}_$r.json 2> $O/b${v}_$r.err || { tail -20 $O/b${v}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b${v}_$r.json')); print('in_block=$v', d['value'], d['ms_per_step'])"
  done
done
bash $R/tools/gpu_r04_prof3.sh r04v | tail -3
