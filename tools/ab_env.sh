#!/bin/bash
# A/B one library under two environments: bench (headline, no gen) + kernel stats + one step's
# timeline per arm.  Usage: bash tools/ab_env.sh TAG "VAR=a" "VAR=b"
set -o pipefail
TAG=$1; A=$2; B=$3
export TMPDIR=/tmp
for arm in a b; do
  E=$A; [ $arm = b ] && E=$B
  env $E timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --no-gen > gpurun_out/abe_${TAG}_$arm.json 2>/dev/null || { echo "bench $arm failed"; exit 1; }
done
for arm in a b; do
  E=$A; [ $arm = b ] && E=$B
  env $E timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --no-gen > gpurun_out/abe_${TAG}_${arm}2.json 2>/dev/null || { echo "bench $arm failed"; exit 1; }
done
echo abe ok
