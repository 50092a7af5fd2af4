#!/bin/bash
# parity subset + step A/B + rocprof timelines: default vs a variant build.  Usage: VARIANT TESTS_K
set -o pipefail
mkdir -p gpurun_out
V=$1; K=${2:-"plan or embed or pre"}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py -k "$K" > gpurun_out/pytest_var2.log 2>&1 || { tail -30 gpurun_out/pytest_var2.log; exit 1; }
tail -2 gpurun_out/pytest_var2.log
CONFIGS="arch3:8" bash tools/ab_env.sh "-" "LBWN_LIB=lb-wavenet_amd/lbwn/abl/liblbwn_g$V.so" > gpurun_out/ab_var2.txt 2>&1 || { cat gpurun_out/ab_var2.txt; exit 1; }
cat gpurun_out/ab_var2.txt
bash tools/gpu_prof_ab.sh $V > gpurun_out/pab_var2.txt 2>&1 || exit 1
cat gpurun_out/pab_var2.txt
