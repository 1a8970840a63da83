#!/bin/bash
# same-box A/B: the tree before the keep-bits change (tools/bin/oldtree, commit 8378ecd) vs now
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04p
mkdir -p $O
R=$GRAFT_REPO_ROOT
for r in 1 2; do
  (cd $R/tools/bin/oldtree && PYTHONPATH=$R/tools/bin/oldtree timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-lm --no-f32 > $O/old_$r.json 2> $O/old_$r.err) || { tail -20 $O/old_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/old_$r.json')); print('old', d['value'], d['ms_per_step'])"
  (cd $R && PYTHONPATH=$R timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-lm --no-f32 > $O/new_$r.json 2> $O/new_$r.err) || { tail -20 $O/new_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/new_$r.json')); print('new', d['value'], d['ms_per_step'])"
done
