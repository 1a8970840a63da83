#!/bin/bash
# round-5 closing pass: every GPU test, smoke(), the default bench command (fp32 C2 headline + the
# bf16 C2 / C4 SOAP / C4 Shampoo / LM 124M / LM 420M sub-lines, each with roofline and CPU baseline),
# with its wall time
set -o pipefail
TAG=${1:-r05z}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export PYTHONPATH=$R
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --tb=short --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/tests.log | head -20
tail -1 $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
s0=$(date +%s)
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo "default bench wall $(( $(date +%s) - s0 )) s"
python - <<PY
import json
d = json.load(open("$O/bench.json"))
print("headline", d["config"]["workload"][:40], d["value"], d["ms_per_step"], "frac", d["roofline"]["frac"], "cpu", d["cpu_baseline"]["value"])
for k, v in d.items():
    if isinstance(v, dict) and "value" in v and "metric" in v:
        print(k, v["value"], v.get("ms_per_step"), "frac", (v.get("roofline") or {}).get("frac"), "cpu", (v.get("cpu_baseline") or {}).get("value"))
PY
