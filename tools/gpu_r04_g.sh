#!/bin/bash
# round 4: tests after the key-owned attention backward + embed+LN fix, phase stamps, then the C2 A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04g
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_vit_parity_gpu.py tests/test_engine_parity_gpu.py tests/test_golden.py -m gpu -x -v -s --tb=short --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -8
[ $rc -ne 0 ] && exit $rc
PLAINCV_HIP_LIB=$GRAFT_REPO_ROOT/tools/bin/v/libsh.so timeout -k 10 120 python tools/sh_phases.py > $O/sh_phases.txt 2>&1 || { tail -20 $O/sh_phases.txt; exit 1; }
cat $O/sh_phases.txt
PCV_ATTN_BWD_TWO_PASS=1 PLAINCV_HIP_LIB=$GRAFT_REPO_ROOT/tools/bin/v/libsh.so timeout -k 10 120 python tools/sh_phases.py > $O/sh_phases_two_pass.txt 2>&1 || { tail -20 $O/sh_phases_two_pass.txt; exit 1; }
grep bwd $O/sh_phases_two_pass.txt
run() {   # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-lm --no-f32 > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$tag.json')); print('$tag', d['value'], d['ms_per_step'], d['config'].get('optimizer_overlap'))"
}
for rep in 1 2; do
  run base_$rep X=1
  run twopass_$rep PCV_ATTN_BWD_TWO_PASS=1
  run nooverlap_$rep PCV_BENCH_OPT_OVERLAP=0
  run nodeltagemm_$rep PCV_VIT_DELTA_GEMM=0
  run noembedln_$rep PCV_VIT_EMBED_LN=0
done
