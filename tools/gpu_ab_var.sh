#!/bin/bash
# Parity subset for the chains + same-box A/B of the default library against a variant build.
# Usage: bash tools/gpu_ab_var.sh VARIANT [CONFIGS]
set -o pipefail
mkdir -p gpurun_out
V=$1; CONFIGS=${2:-"arch3:8 arch5:8"}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py -k "chain or plan or arch5 or full_size" > gpurun_out/pytest_var.log 2>&1 || { tail -30 gpurun_out/pytest_var.log; exit 1; }
tail -2 gpurun_out/pytest_var.log
CONFIGS="$CONFIGS" bash tools/ab_env.sh "-" "LBWN_LIB=lb-wavenet_amd/lbwn/abl/liblbwn_g$V.so" > gpurun_out/ab_var.txt 2>&1 || { cat gpurun_out/ab_var.txt; exit 1; }
cat gpurun_out/ab_var.txt
