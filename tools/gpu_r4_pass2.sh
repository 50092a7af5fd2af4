#!/bin/bash
# Round-4 second pass: PMC traffic for C4 / C5 (sub-benchmark rooflines), dZ read-request split,
# and same-box A/Bs of the chains' XCD-grouped tile walk and dZ's 2-D XCD blocking.
# Usage: bash tools/gpu_r4_pass2.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4}
TAG=c4 bash tools/pmc_traffic.sh --arch par/arch5.json --batch 32 > gpurun_out/pmc_traffic_c4_$TAG.log 2>&1 || exit 1
TAG=c5 bash tools/pmc_traffic.sh --arch par/arch5.json --batch 8 > gpurun_out/pmc_traffic_c5_$TAG.log 2>&1 || exit 1
bash tools/pmc_req.sh > gpurun_out/pmc_req_$TAG.log 2>&1 || exit 1
CONFIGS="arch3:8 arch5:8" bash tools/ab_env.sh "LBWN_CHAIN_XCD=0 LBWN_DZ_XCD=0" "LBWN_CHAIN_XCD=1 LBWN_DZ_XCD=0" "LBWN_CHAIN_XCD=1 LBWN_DZ_XCD=1" > gpurun_out/ab_xcd_$TAG.txt 2>&1 || exit 1
echo pass2 ok
