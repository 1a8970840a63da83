#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04d
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python tools/rp_phases.py > $O/rp_times.txt 2>&1 || { tail -20 $O/rp_times.txt; exit 1; }
echo "== register staging"; grep -v amdgpu.ids $O/rp_times.txt
PLAINCV_HIP_LIB=$GRAFT_REPO_ROOT/scratch/v/librpdma.so timeout -k 10 300 python tools/rp_phases.py > $O/rp_times_dma.txt 2>&1 || { tail -20 $O/rp_times_dma.txt; exit 1; }
echo "== LDS-DMA staging"; grep -v amdgpu.ids $O/rp_times_dma.txt
PLAINCV_HIP_LIB=$GRAFT_REPO_ROOT/scratch/v/libgtime.so timeout -k 10 300 python tools/rp_phases.py --stamps > $O/rp_stamps.txt 2>&1 || { tail -20 $O/rp_stamps.txt; exit 1; }
grep -v amdgpu.ids $O/rp_stamps.txt | tail -10
