#!/bin/bash
# One GPU iteration: parity tests, bench line, rocprof kernel stats + one step's timeline.
# Usage (on the box):  bash tools/gpu_cycle.sh TAG [bench args...]   (TESTS=0 skips the tests)
set -o pipefail
TAG=${1:-x}; shift
mkdir -p gpurun_out
if [ "${TESTS:-1}" != "0" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_$TAG.log; exit 1; }
  tail -2 gpurun_out/t_$TAG.log
fi
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 10 --no-cpu-baseline --no-extras --gen-seconds 0.25 "$@" > gpurun_out/prof_$TAG.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
S=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)
[ -n "$S" ] && python tools/prof_summary.py "$S" gpurun_out/stats_$TAG.md 18 "$TAG" || true
T=$(find gpurun_out/prof_$TAG -name '*kernel_trace.csv' | head -1)
[ -n "$T" ] && python tools/step_timeline.py "$T" > gpurun_out/timeline_$TAG.txt 2>&1 || true
echo "cycle $TAG ok"
