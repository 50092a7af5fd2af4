#!/bin/bash
# rocprof kernel stats + one step's timeline at C4 (arch5 B=32) and C5 per GPU (arch5 B=8).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4}
for cfg in 32 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_a5b${cfg}_$TAG -o run -- \
    python bench.py --arch par/arch5.json --batch $cfg --steps 12 --warmup 3 --no-gen --no-cpu-baseline --no-extras \
    > gpurun_out/prof_a5b${cfg}_$TAG.log 2>&1 || exit 1
  S=$(find gpurun_out/prof_a5b${cfg}_$TAG -name '*kernel_stats.csv' | head -1)
  python tools/prof_summary.py "$S" gpurun_out/stats_a5b${cfg}_$TAG.md 15 a5b${cfg}_$TAG
  K=$(find gpurun_out/prof_a5b${cfg}_$TAG -name '*kernel_trace.csv' | head -1)
  python tools/step_timeline.py "$K" 8 > gpurun_out/timeline_a5b${cfg}_$TAG.txt 2>&1
  echo "== arch5 B=$cfg"; cat gpurun_out/timeline_a5b${cfg}_$TAG.txt
done
