#!/bin/bash
# One GPU iteration: parity tests, bench line, rocprof kernel stats.  Usage (on the box):
#   bash tools/gpu_cycle.sh TAG [bench args...]
set -o pipefail
TAG=${1:-x}; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_$TAG.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 10 --no-cpu-baseline --gen-seconds 0.25 "$@" > gpurun_out/prof_$TAG.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
echo "cycle $TAG ok"
