#!/bin/bash
# HBM bytes and L2 hit rate of one GEMM shape (tools/gemm_one.py), one rocprofv3 --pmc pass per
# counter group, each under its own kill timeout:  tools/gemm_mem.sh TAG "KIND M N K reps"
TAG=${1:?tag}; WL=${2:?"KIND M N K reps"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
db() { ls "$1"/*.db "$1"/*/*.db 2>/dev/null | head -1; }
pass() {   # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $O/$name -o p -- python3 $R/tools/gemm_one.py $WL > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass hit TCC_HIT_sum TCC_MISS_sum
(cd $R/profiles && python3 pmc_traffic.py "$(db $O/fetch)" "$(db $O/write)" "gemm" $O/traffic.json) > $O/traffic.txt 2>&1
(cd $R/profiles && python3 - "$(db $O/hit)" <<'PY'
import sys
from mfma_util import load
per, meta = load(sys.argv[1])
h = m = 0.0
for d, c in per.items():
    h += c.get("TCC_HIT_sum", 0.0); m += c.get("TCC_MISS_sum", 0.0)
print(f"L2 hit {h:.4g} miss {m:.4g} hit rate {h / max(h + m, 1):.3f} (all dispatches)")
PY
) >> $O/traffic.txt 2>&1
rm -rf $O/fetch $O/write $O/hit
cat $O/traffic.txt
