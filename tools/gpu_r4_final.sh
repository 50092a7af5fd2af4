#!/bin/bash
# Round-4 closing pass at HEAD: tests + smoke + bench + C2 profiles (gpu_r4_full.sh), then the arch5
# PMC traffic (C4 = B=32, C5 per GPU = B=8) and the arch5 timelines.  Usage: TAG
set -o pipefail
TAG=${1:-r04_final}
bash tools/gpu_r4_full.sh $TAG || exit 1
TAG=c4 bash tools/pmc_traffic.sh --arch par/arch5.json --batch 32 > gpurun_out/pmc_traffic_c4_$TAG.log 2>&1 || { tail -5 gpurun_out/pmc_traffic_c4_$TAG.log; exit 1; }
TAG=c5 bash tools/pmc_traffic.sh --arch par/arch5.json --batch 8 > gpurun_out/pmc_traffic_c5_$TAG.log 2>&1 || { tail -5 gpurun_out/pmc_traffic_c5_$TAG.log; exit 1; }
bash tools/gpu_prof_c4.sh $TAG > gpurun_out/prof_c4_$TAG.txt 2>&1 || { tail -5 gpurun_out/prof_c4_$TAG.txt; exit 1; }
echo final ok
