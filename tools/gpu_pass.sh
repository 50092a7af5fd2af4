#!/bin/bash
# Measurement pass at HEAD (GPU box): the -m gpu suite, smoke, the full bench line, rocprof
# kernel stats + one step's timeline (C2, C4, C5 per GPU), chain and generation traces, PMC
# traffic (C2 / C4 / C5) and MFMA-busy passes (C2 / C4 / generation).
# Usage: bash tools/gpu_pass.sh TAG [skip-tests]      (outputs under gpurun_out/)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pass}
if [ "$2" != "skip-tests" ]; then
  bash tools/gpu_tests.sh $TAG || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
fi
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
echo bench ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 10 --no-gen --no-cpu-baseline --no-extras > gpurun_out/prof_$TAG.log 2>&1 || exit 1
S=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)
python tools/prof_summary.py "$S" gpurun_out/stats_$TAG.md 20 $TAG
K=$(find gpurun_out/prof_$TAG -name '*kernel_trace.csv' | head -1)
python tools/step_timeline.py "$K" > gpurun_out/timeline_$TAG.txt 2>&1
bash tools/gpu_prof_c4.sh $TAG > gpurun_out/prof_c4_$TAG.txt 2>&1 || { tail -5 gpurun_out/prof_c4_$TAG.txt; exit 1; }
timeout -k 10 120 python tools/chain_trace.py > gpurun_out/chaintrace_$TAG.txt 2>&1 || exit 1
timeout -k 10 120 python tools/gen_trace.py 10 > gpurun_out/gentrace_$TAG.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gen_$TAG -o run -- python tools/gen_bench.py --batch 10 --steps 4000 > gpurun_out/prof_gen_$TAG.log 2>&1 || exit 1
S=$(find gpurun_out/prof_gen_$TAG -name '*kernel_stats.csv' | head -1)
python tools/prof_summary.py "$S" gpurun_out/stats_gen_$TAG.md 10 gen_$TAG
TAG= bash tools/pmc_traffic.sh > gpurun_out/pmc_traffic_$TAG.log 2>&1 || exit 1
TAG=c4 bash tools/pmc_traffic.sh --arch par/arch5.json --batch 32 > gpurun_out/pmc_traffic_c4_$TAG.log 2>&1 || exit 1
TAG=c5 bash tools/pmc_traffic.sh --arch par/arch5.json --batch 8 > gpurun_out/pmc_traffic_c5_$TAG.log 2>&1 || exit 1
TAG=c2 bash tools/pmc_mfma.sh train > gpurun_out/pmc_mfma_c2_$TAG.log 2>&1 || exit 1
TAG=c4 bash tools/pmc_mfma.sh train --arch par/arch5.json --batch 32 > gpurun_out/pmc_mfma_c4_$TAG.log 2>&1 || exit 1
TAG=c5 bash tools/pmc_mfma.sh train --arch par/arch5.json --batch 8 > gpurun_out/pmc_mfma_c5_$TAG.log 2>&1 || exit 1
TAG=gen bash tools/pmc_mfma.sh gen > gpurun_out/pmc_mfma_gen_$TAG.log 2>&1 || exit 1
echo pass ok
