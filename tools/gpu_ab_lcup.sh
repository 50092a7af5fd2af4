#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
LBWN_LC_UP=bwdgemm timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_configs.py -k "arch5" > gpurun_out/pytest_lcup.log 2>&1 || { tail -30 gpurun_out/pytest_lcup.log; exit 1; }
tail -2 gpurun_out/pytest_lcup.log
CONFIGS="arch5:8 arch5:32" bash tools/ab_env.sh "-" "LBWN_LC_UP=bwdgemm" "LBWN_LC_UP=gemm" > gpurun_out/ab_lcup.txt 2>&1 || { cat gpurun_out/ab_lcup.txt; exit 1; }
cat gpurun_out/ab_lcup.txt
