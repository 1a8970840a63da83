#!/bin/bash
# sweep the weight-gradient split count (PCV_WGRAD_SPLITS) over the LM wgrad shapes
set -e
for s in 0 5 9; do
  echo "== splits $s"
  PCV_WGRAD_SPLITS=$s PYTHONPATH=. timeout -k 10 100 python tools/gemm_bench.py wgrad --no-ref
done
