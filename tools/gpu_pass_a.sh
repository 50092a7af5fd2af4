#!/bin/bash
# Measurement pass, part 1 (GPU box): the -m gpu suite, smoke, the full bench line, rocprof kernel
# stats + one step's timeline at C2, C4 and C5 per GPU.  Usage: bash tools/gpu_pass_a.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pass}
bash tools/gpu_tests.sh $TAG || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
echo bench ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 10 --no-gen --no-cpu-baseline --no-extras > gpurun_out/prof_$TAG.log 2>&1 || exit 1
S=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)
python tools/prof_summary.py "$S" gpurun_out/stats_$TAG.md 20 $TAG
K=$(find gpurun_out/prof_$TAG -name '*kernel_trace.csv' | head -1)
python tools/step_timeline.py "$K" > gpurun_out/timeline_$TAG.txt 2>&1
bash tools/gpu_prof_c4.sh $TAG > gpurun_out/prof_c4_$TAG.txt 2>&1 || { tail -5 gpurun_out/prof_c4_$TAG.txt; exit 1; }
echo pass-a ok
