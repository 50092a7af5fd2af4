#!/bin/bash
# Measurement pass, part 2 (GPU box): chain and generation traces, generation rocprof, PMC traffic
# (C2 / C4 / C5) and MFMA-busy passes (C2 / C4 / C5 / generation).  Usage: bash tools/gpu_pass_b.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pass}
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
echo pass-b ok
