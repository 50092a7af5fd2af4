#!/bin/bash
# GPU tests, then forward-chain variant traces.  Usage: bash tools/gpu_tests_abl.sh TAG A1 A2 ...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_$TAG.log; exit 1; }
tail -1 gpurun_out/t_$TAG.log
bash tools/fwd_abl.sh "$@"
