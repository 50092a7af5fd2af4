#!/bin/bash
# A/B several environments of one library on one box: the headline bench (no gen) per arm, all
# arms twice, interleaved; prints ms_per_step per arm and round.
# Usage: bash tools/ab_multi.sh TAG "VAR=a [VAR2=b]" "VAR=c" ...   ("-" = no extra env)
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for round in 1 2; do
  i=0
  for E in "$@"; do
    i=$((i + 1))
    [ "$E" = "-" ] && E="LBWN_NOOP=1"
    env $E timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --no-gen > gpurun_out/abm_${TAG}_${i}_$round.json 2>/dev/null || { echo "bench arm $i ($E) failed"; exit 1; }
    echo "$round arm$i [$E] $(python -c "import json,sys;print(json.load(open(sys.argv[1]))['ms_per_step'])" gpurun_out/abm_${TAG}_${i}_$round.json)"
  done
done
echo abm ok
