#!/bin/bash
# round-3 full pass: every GPU test (verbose log), smoke(), then the default bench line
set -o pipefail
TAG=${1:-r03full}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 800 python -u -m pytest tests -m gpu -v --tb=short --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/tests.log | head -20
tail -1 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_vit_c2.json 2> $O/bench_vit_c2.err || exit $?
python -c "import json; d=json.load(open('$O/bench_vit_c2.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['lm124m']['value'])"
