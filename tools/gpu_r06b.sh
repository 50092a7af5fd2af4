#!/bin/bash
# Round 6: same-box A/Bs -- backward chain weight-gradient roles (one owner per tile vs position
# halves), C2 and C4; the GC side-stream kernels at C4.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "plan_forward_backward or conditioning or configs or fullsize" > gpurun_out/t_r06b.log 2>&1 || { tail -30 gpurun_out/t_r06b.log; exit 1; }
tail -2 gpurun_out/t_r06b.log
bash tools/ab_lib.sh roles lb-wavenet_amd/lbwn/abl/liblbwn_ghalves.so || exit 1
bash tools/ab_lib.sh roles5 lb-wavenet_amd/lbwn/abl/liblbwn_ghalves.so lb-wavenet_amd/lbwn/abl/liblbwn_ggc0.so -- --arch par/arch5.json --batch 32 --steps 10 --warmup 4 || exit 1
LBWN_CHAIN_TRACE=1 timeout -k 10 120 python tools/chain_trace.py > gpurun_out/ct_roles.txt 2>&1 || exit 1
sed -n '/chain_bwd_x3/,$p' gpurun_out/ct_roles.txt
echo r06b ok
