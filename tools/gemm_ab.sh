#!/bin/bash
# Same-box A/B of GEMM variants (lb-wavenet_amd/lbwn/abl/liblbwn_g*.so vs the default build):
# C2 bench step (two interleaved rounds) + the GEMM microbench.  Usage: bash tools/gemm_ab.sh v1 v2 ...
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then unset LBWN_LIB; else export LBWN_LIB=lb-wavenet_amd/lbwn/abl/liblbwn_g$v.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --steps 30 > gpurun_out/gab_$v.json 2> gpurun_out/gab_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/gab_$v.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/gab_$v.json')); print('round $round $v', round(d['ms_per_step'],4))"
  done
done
for v in default "$@"; do
  if [ "$v" = default ]; then unset LBWN_LIB; else export LBWN_LIB=lb-wavenet_amd/lbwn/abl/liblbwn_g$v.so; fi
  echo "== gemm_bench $v"
  GEMM_ONLY=skip_fwd,dz,dskip,post1_fwd,ds,dh timeout -k 10 200 python tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
