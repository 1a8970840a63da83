#!/bin/bash
set -o pipefail
TAG=${1:-r05g}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export PYTHONPATH=$R
cd $R
timeout -k 10 300 python tools/overlap_diag5.py > $O/overlap_diag.txt 2>&1; cat $O/overlap_diag.txt | cut -c1-900
timeout -k 10 300 python tools/f32_dense_times.py > $O/f32_dense_times.txt 2>&1 || { tail -20 $O/f32_dense_times.txt; exit 1; }
cat $O/f32_dense_times.txt
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - <<PY
import json
d=json.load(open('$O/bench.json'))
print('headline', d['value'], d['ms_per_step'], d['roofline']['kernel'][:60], d['roofline']['frac'], d['cpu_baseline']['value'])
for k in ('vit_c2_bf16','vit_c4_soap','vit_c4_shampoo','lm124m','lm420m'):
    x=d[k]; print(k, x['value'], x['ms_per_step'], x['roofline']['frac'] if x.get('roofline') else None, (x.get('cpu_baseline') or {}).get('value'))
PY
