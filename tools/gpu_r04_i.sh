#!/bin/bash
# round 4: L2 reuse probe, attention tests (short + LM), short-attention phases, C2 and LM bench lines
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04i
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 120 tools/bin/xcd_probe > $O/xcd_probe.txt 2>&1 || { cat $O/xcd_probe.txt; exit 1; }
cat $O/xcd_probe.txt
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_lm_parity_gpu.py -m gpu -x -q --tb=short --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
PLAINCV_HIP_LIB=$GRAFT_REPO_ROOT/tools/bin/v/libsh.so timeout -k 10 120 python tools/sh_phases.py > $O/sh_phases.txt 2>&1 || { tail -20 $O/sh_phases.txt; exit 1; }
grep -v amdgpu.ids $O/sh_phases.txt
for rep in 1 2; do
  for x in 0 1; do
    if [ $x = 1 ]; then export PCV_ATTN_XCD=1; else unset PCV_ATTN_XCD; fi
    timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-lm --no-f32 > $O/bench_c2_${rep}_$x.json 2> $O/bench_c2_${rep}_$x.err || { tail -20 $O/bench_c2_${rep}_$x.err; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_c2_${rep}_$x.json')); print('c2 attn_xcd=$x', d['value'], d['ms_per_step'])"
  done
done
unset PCV_ATTN_XCD
timeout -k 10 300 python bench.py --workload lm124m --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_lm124m.json 2> $O/bench_lm124m.err || { tail -20 $O/bench_lm124m.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_lm124m.json')); print('lm124m', d['value'], d['ms_per_step'])"
