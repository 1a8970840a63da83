#!/bin/bash
# round 4: instruction-fetch probe, the kernel/engine tests after the embed+LN fix, then the C2 A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04f
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 60 tools/bin/icache_probe > $O/icache_probe.txt 2>&1 || { cat $O/icache_probe.txt; exit 1; }
cat $O/icache_probe.txt
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_parity_gpu.py -m gpu -x -v -s --tb=short --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -8
[ $rc -ne 0 ] && exit $rc
for v in "1 1 1" "0 1 1" "1 0 1" "1 1 0" "1 1 1" "0 1 1" "1 0 1" "1 1 0"; do
  set -- $v
  PCV_BENCH_OPT_OVERLAP=$1 PCV_VIT_DELTA_GEMM=$2 PCV_VIT_EMBED_LN=$3 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-lm --no-f32 > $O/bench_$1$2$3.json 2> $O/bench_$1$2$3.err || { tail -20 $O/bench_$1$2$3.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$1$2$3.json')); print('overlap=$1 delta_gemm=$2 embed_ln=$3', d['value'], d['ms_per_step'], d['config']['optimizer_overlap'])"
done
