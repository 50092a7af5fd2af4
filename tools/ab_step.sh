#!/bin/bash
# Same-box A/B of library variants (lb-wavenet_amd/lbwn/abl/liblbwn_g*.so vs the default build) on
# the training step, two interleaved rounds.  CONFIGS (default "arch3:8 arch5:8"): arch:batch list,
# e.g. "arch5:8 arch5:32" for C5's per-GPU share and C4.  Usage: bash tools/ab_step.sh v1 v2 ...
set -o pipefail
mkdir -p gpurun_out
CONFIGS=${CONFIGS:-"arch3:8 arch5:8"}
for round in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then unset LBWN_LIB; else export LBWN_LIB=lb-wavenet_amd/lbwn/abl/liblbwn_g$v.so; fi
    for cfg in $CONFIGS; do
      arch=${cfg%%:*}; b=${cfg#*:}
      steps=30; [ "$b" -gt 8 ] && steps=10
      timeout -k 10 240 python bench.py --arch par/$arch.json --batch $b --no-cpu-baseline --no-extras --no-gen \
        --steps $steps > gpurun_out/abs_${v}_$arch$b.json 2> gpurun_out/abs_${v}_$arch$b.err || { echo "bench $v $cfg failed"; tail -5 gpurun_out/abs_${v}_$arch$b.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/abs_${v}_$arch$b.json')); print('round $round $v $cfg', round(d['ms_per_step'],4), 'fwd', round(d['roofline_dilconv']['avg_launch_us'],1), 'bwd', round(d['roofline']['avg_launch_us'],1))"
    done
  done
done
