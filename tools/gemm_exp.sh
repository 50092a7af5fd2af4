#!/bin/bash
# GEMM microbench only (no training step) over library variants: for timing-only experiment
# builds whose results are wrong.  Usage: bash tools/gemm_exp.sh v1 v2 ...  (GEMM_ONLY honoured)
set -o pipefail
for v in default "$@"; do
  if [ "$v" = default ]; then unset LBWN_LIB; else export LBWN_LIB=lb-wavenet_amd/lbwn/abl/liblbwn_g$v.so; fi
  echo "== gemm_bench $v"
  timeout -k 10 200 python tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
