#!/bin/bash
# A/B k-tile ring depth variants of the 128x128 / 64x64 GEMM family (plaincv_amd/libplaincv_hip_<v>.so)
set -e
export PYTHONPATH=$PWD
for v in base ${@:-g3 g4 b3 s3}; do
  L=$PWD/plaincv_amd/libplaincv_hip.so
  [ "$v" != base ] && L=$PWD/plaincv_amd/libplaincv_hip_$v.so
  echo "== $v $(PLAINCV_HIP_LIB=$L timeout -k 10 100 python bench.py --no-cpu-baseline --steps 100 --warmup 20 2>/dev/null | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  PLAINCV_HIP_LIB=$L timeout -k 10 100 python tools/gemm_bench.py "wgrad" --no-ref --graph 2>/dev/null | grep -v "lm_head" | cut -c1-80
done
