#!/bin/bash
# Round 6: XCD-local hand-offs (plain halo stores to a same-XCD consumer) with the XCD-grouped walk.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "placement or plan_forward_backward or conditioning or chain_matches" > gpurun_out/t_r06e.log 2>&1 || { tail -30 gpurun_out/t_r06e.log; exit 1; }
tail -2 gpurun_out/t_r06e.log
bash tools/ab_env.sh xl "LBWN_CHAIN_XCD=0" "LBWN_CHAIN_XCD=1 LBWN_CHAIN_XLOCAL=1" "LBWN_CHAIN_XCD=1" || exit 1
bash tools/ab_env.sh xl5 "LBWN_CHAIN_XCD=1" "LBWN_CHAIN_XCD=1 LBWN_CHAIN_XLOCAL=1" -- --arch par/arch5.json --batch 32 --steps 10 --warmup 4 || exit 1
LBWN_CHAIN_XCD=1 LBWN_CHAIN_XLOCAL=1 timeout -k 10 120 python tools/chain_trace.py > gpurun_out/ct_xl.txt 2>&1 || exit 1
cat gpurun_out/ct_xl.txt | head -12
echo r06e ok
