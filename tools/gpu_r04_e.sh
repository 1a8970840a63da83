#!/bin/bash
# round 4: ADVICE-driven tests + optimizer-overlap test, the C2 step A/B (optimizer overlap, GEMM delta),
# then the row-panel staging comparison
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04e
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_vit_parity_gpu.py tests/test_dp_gpu.py tests/test_golden.py -m gpu -x -v -s --tb=short --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "SHARD|FAILED|ERROR|passed|failed" $O/tests.log | tail -20
[ $rc -ne 0 ] && exit $rc
for v in "1 1" "0 1" "1 0" "1 1" "0 1" "1 0"; do
  set -- $v
  PCV_BENCH_OPT_OVERLAP=$1 PCV_VIT_DELTA_GEMM=$2 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-lm --no-f32 > $O/bench_$1$2.json 2> $O/bench_$1$2.err || { tail -20 $O/bench_$1$2.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$1$2.json')); print('overlap=$1 delta_gemm=$2', d['value'], d['ms_per_step'], d['config']['optimizer_overlap'])"
done
timeout -k 10 300 python tools/rp_phases.py > $O/rp_times.txt 2>&1 || { tail -20 $O/rp_times.txt; exit 1; }
echo "== register staging"; grep -v amdgpu.ids $O/rp_times.txt
PLAINCV_HIP_LIB=$GRAFT_REPO_ROOT/scratch/v/librpdma.so timeout -k 10 300 python tools/rp_phases.py > $O/rp_times_dma.txt 2>&1 || { tail -20 $O/rp_times_dma.txt; exit 1; }
echo "== LDS-DMA staging"; grep -v amdgpu.ids $O/rp_times_dma.txt
