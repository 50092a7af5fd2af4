#!/bin/bash
# Round-6 A/B: residual-stack weight gradients in the backward chain vs layer_wgrad_kernel.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${WGK:-wg and (plan_forward_backward or conditioning or shorter)}" > gpurun_out/t_wg.log 2>&1 || { tail -40 gpurun_out/t_wg.log; exit 1; }
tail -3 gpurun_out/t_wg.log
bash tools/ab_env.sh wg "LBWN_BWD_WGRAD=0" "LBWN_BWD_WGRAD=1" || exit 1
LBWN_BWD_WGRAD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wg1 -o run -- python bench.py --steps 10 --no-gen --no-cpu-baseline --no-extras > gpurun_out/prof_wg1.log 2>&1 || exit 1
S=$(find gpurun_out/prof_wg1 -name '*kernel_stats.csv' | head -1)
python tools/prof_summary.py "$S" gpurun_out/stats_wg1.md 20 wg1
K=$(find gpurun_out/prof_wg1 -name '*kernel_trace.csv' | head -1)
python tools/step_timeline.py "$K" > gpurun_out/timeline_wg1.txt 2>&1
echo wg ok
