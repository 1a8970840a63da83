#!/bin/bash
# round-4 closing pass: every GPU test, smoke(), the default bench line (+ CPU baseline and the LM
# sub-lines), the C2 kernel table and one step's kernel sequence, the C4 lines.
set -o pipefail
TAG=${1:-r04z}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export PYTHONPATH=$R
timeout -k 10 900 python -u -m pytest tests -m gpu -v --tb=short --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/tests.log | head -20
tail -1 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_vit_c2.json 2> $O/bench_vit_c2.err || { tail -20 $O/bench_vit_c2.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_vit_c2.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['vit_c2_f32']['value'], d['lm124m']['value'])"
