#!/bin/bash
# Round 6: backward chain bias sums folded into the dSIG / dRES operand reads (default build) vs HEAD.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "plan_forward_backward or conditioning or shorter or staged or configs or fullsize" > gpurun_out/t_r06d.log 2>&1 || { tail -30 gpurun_out/t_r06d.log; exit 1; }
tail -2 gpurun_out/t_r06d.log
bash tools/ab_lib.sh fold lb-wavenet_amd/lbwn/abl/liblbwn_ghead.so || exit 1
bash tools/ab_lib.sh fold5 lb-wavenet_amd/lbwn/abl/liblbwn_ghead.so -- --arch par/arch5.json --batch 32 --steps 10 --warmup 4 || exit 1
timeout -k 10 120 python tools/chain_trace.py > gpurun_out/ct_fold.txt 2>&1 || exit 1
sed -n '/chain_bwd_x3/,$p' gpurun_out/ct_fold.txt
echo r06d ok
