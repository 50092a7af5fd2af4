#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "gemm or plan_forward_backward or placement" > gpurun_out/pytest_amn.log 2>&1 || { tail -30 gpurun_out/pytest_amn.log; exit 1; }
tail -2 gpurun_out/pytest_amn.log
GEMM_ONLY=dskip,dpost1,dpost2 timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/gb_amn.txt 2>&1 || { cat gpurun_out/gb_amn.txt; exit 1; }
cat gpurun_out/gb_amn.txt
CONFIGS="arch3:8 arch5:8" bash tools/ab_env.sh "-" "LBWN_GEMM_AMN=0" > gpurun_out/ab_amn.txt 2>&1 || { cat gpurun_out/ab_amn.txt; exit 1; }
cat gpurun_out/ab_amn.txt
