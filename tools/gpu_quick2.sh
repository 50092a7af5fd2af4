#!/bin/bash
# tests + arch3 chain trace + bench cycle (no tests) + arch5 profile
set -o pipefail
TAG=$1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_$TAG.log; exit 1; }
tail -1 gpurun_out/t_$TAG.log
timeout -k 10 120 python tools/chain_trace.py 1 > gpurun_out/ctrace_$TAG.txt 2>&1 || { echo "trace failed"; tail gpurun_out/ctrace_$TAG.txt; exit 1; }
cat gpurun_out/ctrace_$TAG.txt | grep -v amdgpu.ids
TESTS=0 bash tools/gpu_cycle.sh $TAG || exit 1
python -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print('C2 ms', d['ms_per_step'], 'fwd', d['roofline_dilconv']['avg_launch_us'], 'bwd', d['roofline']['avg_launch_us'])"
bash tools/prof_arch.sh a5$TAG par/arch5.json || exit 1
echo "quick2 $TAG ok"
