#!/bin/bash
# A/B the GEMM ring/barrier build variants (plaincv_amd/libplaincv_hip_s*_r*.so) on the LM shapes
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD
for v in ${@:-s2_r0 s2_r1 s3_r1 s4_r1}; do
  echo "== $v"
  PLAINCV_HIP_LIB=$PWD/plaincv_amd/libplaincv_hip_$v.so timeout -k 10 200 python tools/gemm_bench.py fwd --no-ref
  PLAINCV_HIP_LIB=$PWD/plaincv_amd/libplaincv_hip_$v.so timeout -k 10 200 python tools/gemm_bench.py dgrad --no-ref
done
