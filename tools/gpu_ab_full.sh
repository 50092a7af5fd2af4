#!/bin/bash
# full GPU suite + same-box step A/B (arch3 / arch5 B=8, two rounds) against a variant build +
# rocprof timelines of both.  Usage: VARIANT
set -o pipefail
mkdir -p gpurun_out
V=$1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/pytest_abfull.log 2>&1 || { tail -30 gpurun_out/pytest_abfull.log; exit 1; }
tail -2 gpurun_out/pytest_abfull.log
bash tools/ab_env.sh "-" "LBWN_LIB=lb-wavenet_amd/lbwn/abl/liblbwn_g$V.so" > gpurun_out/ab_full.txt 2>&1 || { cat gpurun_out/ab_full.txt; exit 1; }
cat gpurun_out/ab_full.txt
bash tools/gpu_prof_ab.sh $V > gpurun_out/pab_full.txt 2>&1 || exit 1
cat gpurun_out/pab_full.txt
