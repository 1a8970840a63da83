#!/bin/bash
# ViT C2 step time vs grouped weight-gradient tile / block target
set -e
for cfg in "64 1024" "64 512" "64 2048" "128 256" "128 512" "128 1024"; do
  set -- $cfg
  echo "tile $1 blocks $2"
  PCV_WGRAD_TILE=$1 PCV_WGRAD_BLOCKS=$2 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --warmup 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['final_loss'])"
done
