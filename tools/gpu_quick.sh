#!/bin/bash
# Quick GPU check: the full -m gpu suite, then optional profiles.  Usage: bash tools/gpu_quick.sh TAG [prof specs "tag:arch" ...]
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_$TAG.log; exit 1; }
tail -2 gpurun_out/t_$TAG.log
for spec in "$@"; do
  bash tools/prof_arch.sh ${spec%%:*} ${spec#*:} || exit 1
done
echo "quick $TAG ok"
