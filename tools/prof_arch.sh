#!/bin/bash
# rocprof kernel stats + one step's timeline of a training configuration other than C2.
# Usage (on the box): bash tools/prof_arch.sh TAG ARCH_JSON [bench args...]
set -o pipefail
TAG=$1; ARCH=$2; shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --arch $ARCH --steps 10 --warmup 3 --no-cpu-baseline --no-extras --no-gen "$@" > gpurun_out/prof_$TAG.log 2>&1 || { echo "prof $TAG failed"; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
S=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)
[ -n "$S" ] && python tools/prof_summary.py "$S" gpurun_out/stats_$TAG.md 24 "$TAG" || true
T=$(find gpurun_out/prof_$TAG -name '*kernel_trace.csv' | head -1)
[ -n "$T" ] && python tools/step_timeline.py "$T" > gpurun_out/timeline_$TAG.txt 2>&1 || true
tail -1 gpurun_out/prof_$TAG.log
echo "prof $TAG ok"
