#!/bin/bash
# rocprofv3 kernel trace + stats of one bench workload (run through gpurun from the repo root):
#   tools/gpu_prof.sh TAG WORKLOAD STEPS [WARMUP]
# -> gpurun_out/TAG/prof_WORKLOAD/ (rocpd db + stats csv) and gpurun_out/TAG/WORKLOAD_kernel_stats.txt
# (profiles/summarize_rocpd.py over the db; the bench's own roofline / CPU-baseline launches are off).
set -o pipefail
TAG=${1:?tag}; WL=${2:?workload}; STEPS=${3:-5}; WARM=${4:-1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
LMARGS=""
case "$WL" in lm*) LMARGS="--lm-steps $STEPS --lm-warmup $WARM";; esac
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$O/prof_$WL" -o p -- python3 "$R/bench.py" --workload "$WL" \
  --steps "$STEPS" --warmup "$WARM" --no-sub --no-roofline --no-cpu-baseline > "$O/prof_$WL.log" 2>&1 || { tail -20 "$O/prof_$WL.log"; exit 1; }
DB=$(find "$O/prof_$WL" -name "*.db" | head -1)
python3 "$R/profiles/summarize_rocpd.py" "$DB" "$((STEPS + WARM))" > "$O/${WL}_kernel_stats.txt"
head -25 "$O/${WL}_kernel_stats.txt"
