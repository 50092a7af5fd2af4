#!/bin/bash
# Same-box A/B of library variants (lb-wavenet_amd/lbwn/abl/liblbwn_g*.so vs the default build) on
# the training step: C2 (arch3 B=8) and C5's per-GPU share (arch5 B=8), two interleaved rounds.
# Usage: bash tools/ab_step.sh v1 v2 ...
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then unset LBWN_LIB; else export LBWN_LIB=lb-wavenet_amd/lbwn/abl/liblbwn_g$v.so; fi
    for arch in arch3 arch5; do
      timeout -k 10 200 python bench.py --arch par/$arch.json --no-cpu-baseline --no-extras --no-gen --steps 30 \
        > gpurun_out/abs_${v}_$arch.json 2> gpurun_out/abs_${v}_$arch.err || { echo "bench $v $arch failed"; tail -5 gpurun_out/abs_${v}_$arch.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/abs_${v}_$arch.json')); print('round $round $v $arch', round(d['ms_per_step'],4), 'fwd', round(d['roofline_dilconv']['avg_launch_us'],1), 'bwd', round(d['roofline']['avg_launch_us'],1))"
    done
  done
done
