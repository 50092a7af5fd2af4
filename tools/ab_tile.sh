#!/bin/bash
# Same-box A/B of the forward chain forms (LBWN_CHAIN_TILE = w32 / 128 / 64) on the training step,
# two interleaved rounds.  CONFIGS (default "arch3:8 arch5:8"): arch:batch list.
# Usage: bash tools/ab_tile.sh [tiles...]
set -o pipefail
mkdir -p gpurun_out
CONFIGS=${CONFIGS:-"arch3:8 arch5:8"}
TILES=${*:-"w32 128 64"}
for round in 1 2; do
  for v in $TILES; do
    for cfg in $CONFIGS; do
      arch=${cfg%%:*}; b=${cfg#*:}
      steps=30; [ "$b" -gt 8 ] && steps=10
      LBWN_CHAIN_TILE=$v timeout -k 10 240 python bench.py --arch par/$arch.json --batch $b --no-cpu-baseline --no-extras --no-gen \
        --steps $steps > gpurun_out/abt_${v}_$arch$b.json 2> gpurun_out/abt_${v}_$arch$b.err || { echo "bench $v $cfg failed"; tail -5 gpurun_out/abt_${v}_$arch$b.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/abt_${v}_$arch$b.json')); print('round $round tile $v $cfg', round(d['ms_per_step'],4), 'fwd', round(d['roofline_dilconv']['avg_launch_us'],1), 'bwd', round(d['roofline']['avg_launch_us'],1))"
    done
  done
done
