#!/bin/bash
# Same-box A/B of the arch5 backward tail: dLCcat after dlc (default) vs beside it, and dlc's split-K.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_configs.py -k "arch5" > gpurun_out/pytest_lc.log 2>&1 || { tail -20 gpurun_out/pytest_lc.log; exit 1; }
tail -2 gpurun_out/pytest_lc.log
CONFIGS="arch5:8 arch5:32" bash tools/ab_env.sh "-" "LBWN_LC_TAIL=0" "LBWN_DLC_SPLIT=1" "LBWN_DLC_SPLIT=4" > gpurun_out/ab_lc.txt 2>&1 || { cat gpurun_out/ab_lc.txt; exit 1; }
cat gpurun_out/ab_lc.txt
