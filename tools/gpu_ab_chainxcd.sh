#!/bin/bash
# the LC-arch XCD-walk default: bitwise tests + same-box A/B (C4, C5 per GPU, C2 as the control)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "chain_xcd or placement" > gpurun_out/pytest_cx.log 2>&1 || { tail -30 gpurun_out/pytest_cx.log; exit 1; }
tail -2 gpurun_out/pytest_cx.log
CONFIGS="arch5:32 arch5:8 arch3:8" bash tools/ab_env.sh "-" "LBWN_CHAIN_XCD=0" > gpurun_out/ab_cx.txt 2>&1 || { cat gpurun_out/ab_cx.txt; exit 1; }
cat gpurun_out/ab_cx.txt
