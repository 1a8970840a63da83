#!/bin/bash
# Profiles of one bench workload (run through gpurun from the repo root):
#   tools/gpu_profile.sh TAG WORKLOAD STEPS "kernel substring" ["kernel substring" ...]
# 1. HBM bytes per launch of each named kernel: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in
#    separate passes (MI355X_MICROARCH.md HBM section) -> TAG_WORKLOAD_pmc_traffic.{json,txt}
#    (bench.py's `traffic` field reads the newest profiles/r*_pmc_traffic.json);
# 2. MFMA busy / MFMA instruction passes -> TAG_WORKLOAD_mfma_util.txt;
# 3. a kernel-trace pass -> TAG_WORKLOAD_kernel_stats.txt (+ one step's kernel sequence for the ViT).
# Every pass runs under its own kill timeout; the databases are summarised on the box and removed.
set -o pipefail
TAG=${1:?tag}; WL=${2:?workload}; STEPS=${3:-3}; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
db() { ls "$1"/*.db "$1"/*/*.db 2>/dev/null | head -1; }
ARGS="--workload $WL --steps $STEPS --warmup 1 --no-sub --no-cpu-baseline --no-roofline"
case "$WL" in lm*) ARGS="$ARGS --lm-accum 2";; esac
pass() {   # name counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" -d "$O/$name" -o p -- python3 "$R/bench.py" $ARGS > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
P=$O/${TAG}_${WL}
if [ $# -gt 0 ]; then
  pass pmc_fetch FETCH_SIZE
  pass pmc_write WRITE_SIZE
  rm -f "${P}_pmc_traffic.json"
  for k in "$@"; do
    echo "== $k"
    (cd "$R/profiles" && python3 pmc_traffic.py "$(db "$O/pmc_fetch")" "$(db "$O/pmc_write")" "$k" "${P}_pmc_traffic.json") || exit 1
  done > "${P}_pmc_traffic.txt"
  rm -rf "$O/pmc_fetch" "$O/pmc_write"
  cat "${P}_pmc_traffic.txt"
fi
pass busy SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
pass insts SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_WAVE_CYCLES
python3 "$R/profiles/mfma_util.py" "$(db "$O/busy")" "$(db "$O/insts")" "${P}_mfma_util.txt" --top 30 > /dev/null || exit 1
rm -rf "$O/busy" "$O/insts"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o p -- python3 "$R/bench.py" $ARGS > "$O/prof.log" 2>&1 || { tail -20 "$O/prof.log"; exit 1; }
d=$(db "$O/prof")
python3 "$R/profiles/summarize_rocpd.py" "$d" $((STEPS + 1)) > "${P}_kernel_stats.txt" || exit 1
case "$WL" in vit*) python3 "$R/profiles/step_timeline.py" "$d" > "${P}_step_timeline.txt" || exit 1;; esac
rm -rf "$O/prof"
head -20 "${P}_kernel_stats.txt"
head -25 "${P}_mfma_util.txt"
