#!/bin/bash
# SQ counters of one fp32 row-GEMM launch shape (tools/panel_probe.py --only NAME --loop 200, tiled form)
set -o pipefail
NAME=${1:-fc1_d}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05r_$NAME
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS -d $O/pmc -o p --output-format csv -- python3 $R/tools/panel_probe.py --only $NAME --loop 200 --form pcv_gemm_f32_rows_tiled > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
f=$(ls $O/pmc/*counter_collection.csv $O/pmc/*/*counter_collection.csv 2>/dev/null | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for r in csv.DictReader(open(sys.argv[1])):
    if "gemm_f32_rows_kernel" in r["Kernel_Name"]:
        acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"][:80]
n = len(acc)
tot = collections.defaultdict(float)
for d, cs in acc.items():
    for c, v in cs.items():
        tot[c] += v
print(next(iter(names.values())) if names else "-", "dispatches", n)
for c, v in sorted(tot.items()):
    print(f"{c:28s} {v / n:16.0f}")
PY
rm -rf $O/pmc
