#!/bin/bash
# SQ counters of the LM flash-attention kernels at the 124M shape (tools/attn_bench.py lm124m), per wave
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/lmattn_pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $O/$name -o p --output-format csv -- python3 $R/tools/attn_bench.py lm124m > $O/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -ge 124 ] && exit $rc; return 0
}
pass a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU_MFMA_BF16 SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_WAVE_CYCLES
pass b SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS
for n in a b; do
  f=$(ls $O/$n/*counter_collection.csv $O/$n/*/*counter_collection.csv 2>/dev/null | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k = r.get("Kernel_Name", r.get("Kernel-Name", ""))
    if "attn_" not in k:
        continue
    agg[k[:48]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    w = sum(cs.get("SQ_WAVES", [1])) or 1
    print(k, {c: round(sum(v) / w, 1) for c, v in sorted(cs.items()) if c != "SQ_WAVES"})
PY
done
rm -rf $O/a $O/b
