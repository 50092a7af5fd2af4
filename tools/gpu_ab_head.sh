#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "head or plan_forward_backward or colsum or bias" > gpurun_out/pytest_head.log 2>&1 || { tail -30 gpurun_out/pytest_head.log; exit 1; }
tail -2 gpurun_out/pytest_head.log
CONFIGS="arch3:8" bash tools/ab_env.sh "-" "LBWN_LIB=lb-wavenet_amd/lbwn/abl/liblbwn_gprehead.so" > gpurun_out/ab_head.txt 2>&1 || { cat gpurun_out/ab_head.txt; exit 1; }
cat gpurun_out/ab_head.txt
bash tools/gpu_prof_ab.sh prehead > gpurun_out/pab_head.txt 2>&1 || exit 1
grep -E "head_reg|colsum_final|==" gpurun_out/pab_head.txt
