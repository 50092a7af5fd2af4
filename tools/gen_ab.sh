#!/bin/bash
# Same-box A/B of generation variants (lb-wavenet_amd/lbwn/abl/liblbwn_g*.so vs the default build):
# us/step of cached generation at B=10, two interleaved rounds.  Usage: bash tools/gen_ab.sh v1 v2 ...
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then unset LBWN_LIB; else export LBWN_LIB=lb-wavenet_amd/lbwn/abl/liblbwn_g$v.so; fi
    echo -n "round $round $v: "
    timeout -k 10 200 python tools/gen_bench.py --batch 10 --steps 4000 2>&1 | grep -v amdgpu.ids | tail -1 || { echo "gen $v failed"; exit 1; }
  done
done
