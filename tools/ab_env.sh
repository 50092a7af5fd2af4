#!/bin/bash
# Same-box A/B of environment settings on the training step, two interleaved rounds.
# Usage: bash tools/ab_env.sh "LBWN_CHAIN_XCD=0" "LBWN_CHAIN_XCD=1" ...   ("-" = no setting)
# CONFIGS (default "arch3:8 arch5:8"): arch:batch list.
set -o pipefail
mkdir -p gpurun_out
CONFIGS=${CONFIGS:-"arch3:8 arch5:8"}
for round in 1 2; do
  k=0
  for v in "$@"; do
    k=$((k + 1))
    for cfg in $CONFIGS; do
      arch=${cfg%%:*}; b=${cfg#*:}
      steps=40; [ "$b" -gt 8 ] && steps=12
      envs=(); [ "$v" != "-" ] && envs=($v)
      env "${envs[@]}" timeout -k 10 240 python bench.py --arch par/$arch.json --batch $b --no-cpu-baseline --no-extras --no-gen \
        --steps $steps > gpurun_out/abe_${k}_$arch$b.json 2> gpurun_out/abe_${k}_$arch$b.err || { echo "bench [$v] $cfg failed"; tail -5 gpurun_out/abe_${k}_$arch$b.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/abe_${k}_$arch$b.json')); print('round $round [$v] $cfg', round(d['ms_per_step'],4), 'fwd', round(d['roofline_dilconv']['avg_launch_us'],1), 'bwd', round(d['roofline']['avg_launch_us'],1))"
    done
  done
done
