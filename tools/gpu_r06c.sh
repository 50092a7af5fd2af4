#!/bin/bash
# Round 6: backward chain tail -- producer flag read early (default build) vs HEAD vs + bias sums first.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "plan_forward_backward or conditioning or shorter or staged" > gpurun_out/t_r06c.log 2>&1 || { tail -30 gpurun_out/t_r06c.log; exit 1; }
tail -2 gpurun_out/t_r06c.log
bash tools/ab_lib.sh flag lb-wavenet_amd/lbwn/abl/liblbwn_ghead.so lb-wavenet_amd/lbwn/abl/liblbwn_gbiasfirst.so || exit 1
bash tools/ab_lib.sh flag5 lb-wavenet_amd/lbwn/abl/liblbwn_ghead.so lb-wavenet_amd/lbwn/abl/liblbwn_gbiasfirst.so -- --arch par/arch5.json --batch 32 --steps 10 --warmup 4 || exit 1
timeout -k 10 120 python tools/chain_trace.py > gpurun_out/ct_flag.txt 2>&1 || exit 1
sed -n '/chain_bwd_x3/,$p' gpurun_out/ct_flag.txt
timeout -k 10 120 python tools/with_lib.py lb-wavenet_amd/lbwn/abl/liblbwn_gbiasfirst.so tools/chain_trace.py > gpurun_out/ct_biasfirst.txt 2>&1 || exit 1
sed -n '/chain_bwd_x3/,$p' gpurun_out/ct_biasfirst.txt
echo r06c ok
