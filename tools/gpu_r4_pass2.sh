#!/bin/bash
# Round-4 second pass: PMC traffic for C4 / C5 (sub-benchmark rooflines), dZ read-request split,
# and dZ's 2-D XCD blocking (time A/B and traffic without it).
# Usage: bash tools/gpu_r4_pass2.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4}
TAG=c4 bash tools/pmc_traffic.sh --arch par/arch5.json --batch 32 > gpurun_out/pmc_traffic_c4_$TAG.log 2>&1 || exit 1
TAG=c5 bash tools/pmc_traffic.sh --arch par/arch5.json --batch 8 > gpurun_out/pmc_traffic_c5_$TAG.log 2>&1 || exit 1
bash tools/pmc_req.sh > gpurun_out/pmc_req_$TAG.log 2>&1 || exit 1
CONFIGS="arch3:8" bash tools/ab_env.sh "-" "LBWN_DZ_XCD=0" > gpurun_out/ab_dzxcd_$TAG.txt 2>&1 || exit 1
TAG=dz0 LBWN_DZ_XCD=0 bash tools/pmc_traffic.sh > gpurun_out/pmc_traffic_dz0_$TAG.log 2>&1 || exit 1
echo pass2 ok
