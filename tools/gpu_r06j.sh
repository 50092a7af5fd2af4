#!/bin/bash
# Round 6: DP device path host cost (enqueue time per step) with cached bucket views.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r06j.log 2>&1 || { tail -30 gpurun_out/t_r06j.log; exit 1; }
tail -1 gpurun_out/t_r06j.log
timeout -k 10 300 python tools/dp_overhead.py > gpurun_out/dp_c2_j.json 2> gpurun_out/dp_c2_j.err || { tail -20 gpurun_out/dp_c2_j.err; exit 1; }
cat gpurun_out/dp_c2_j.json
timeout -k 10 300 python tools/dp_overhead.py --steps 40 > gpurun_out/dp_c2_j2.json 2> gpurun_out/dp_c2_j2.err || { tail -20 gpurun_out/dp_c2_j2.err; exit 1; }
cat gpurun_out/dp_c2_j2.json
echo r06j ok
