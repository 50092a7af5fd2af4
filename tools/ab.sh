#!/bin/bash
# A/B two library builds on the box: bench (headline, no gen) + backward-chain trace + kernel stats.
# Usage: bash tools/ab.sh TAG VARIANT_SO   (VARIANT_SO relative to lb-wavenet_amd/lbwn/)
set -o pipefail
TAG=$1; V=$2
export TMPDIR=/tmp
for arm in base var; do
  if [ $arm = var ]; then export LBWN_LIB=$PWD/lb-wavenet_amd/lbwn/$V; else unset LBWN_LIB; fi
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --no-gen > gpurun_out/ab_${TAG}_$arm.json 2>/dev/null || { echo "bench $arm failed"; exit 1; }
  timeout -k 10 120 python tools/chain_trace.py 1 > gpurun_out/ab_${TAG}_${arm}_ctrace.txt 2>&1 || { echo "trace $arm failed"; exit 1; }
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_${TAG}_${arm}_prof -o run -- python bench.py --steps 10 --warmup 4 --no-cpu-baseline --no-extras --no-gen > /dev/null 2>&1 || { echo "prof $arm failed"; exit 1; }
done
echo ab ok
