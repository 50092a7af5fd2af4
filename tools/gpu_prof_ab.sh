#!/bin/bash
# Per-kernel rocprof comparison of the default library and a variant build (same box).
# Usage: bash tools/gpu_prof_ab.sh VARIANT_NAME [extra env for the variant, e.g. LBWN_CHAIN_XCD=0]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$1; shift
for which in default $V; do
  if [ $which = default ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pab_$which -o run -- \
      python bench.py --steps 10 --no-gen --no-cpu-baseline --no-extras > gpurun_out/pab_$which.log 2>&1 || exit 1
  else
    env LBWN_LIB=lb-wavenet_amd/lbwn/abl/liblbwn_g$V.so "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      --output-format csv -d gpurun_out/pab_$which -o run -- \
      python bench.py --steps 10 --no-gen --no-cpu-baseline --no-extras > gpurun_out/pab_$which.log 2>&1 || exit 1
  fi
  S=$(find gpurun_out/pab_$which -name '*kernel_stats.csv' | head -1)
  python tools/prof_summary.py "$S" gpurun_out/pab_stats_$which.md 30 $which
  K=$(find gpurun_out/pab_$which -name '*kernel_trace.csv' | head -1)
  python tools/step_timeline.py "$K" > gpurun_out/pab_timeline_$which.txt 2>&1
  echo "== $which"; cat gpurun_out/pab_timeline_$which.txt
done
