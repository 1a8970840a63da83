#!/bin/bash
# row GEMM forms: per-launch timings (tail / no tail, epilogue / plain) + issue/stall PMC per form
set -o pipefail
TAG=${1:-r05l}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export PYTHONPATH=$R
cd $R
timeout -k 10 300 python -u tools/panel_probe.py > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
cat $O/probe.txt
bash tools/pmc_stall.sh $TAG/pmc_panel "--loop 40" tools/panel_probe.py || exit 1
bash tools/pmc_stall.sh $TAG/pmc_tiled "--loop 40 --form pcv_gemm_f32_rows_tiled" tools/panel_probe.py || exit 1
cut -c1-60,61-250 $O/pmc_panel/summary.txt | head -14
cut -c1-60,61-250 $O/pmc_tiled/summary.txt | head -14
