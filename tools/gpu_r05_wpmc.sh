#!/bin/bash
# SQ counters of the fp32 wgrad kernel (one pass, kernel-trace only)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05w
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS -d $O/pmc -o p --output-format csv -- python3 $R/tools/wgrad_sweep.py 768 > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
f=$(ls $O/pmc/*counter_collection.csv $O/pmc/*/*counter_collection.csv 2>/dev/null | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    if "wgrad_kernel" in r["Kernel_Name"]:
        acc[r["Dispatch_Id"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
tot = collections.defaultdict(float)
for d, cs in acc.items():
    for c, v in cs.items():
        tot[c] += sum(v)
n = len(acc)
for c, v in sorted(tot.items()):
    print(f"{c:28s} {v / n:16.0f}")
print("dispatches", n)
PY
