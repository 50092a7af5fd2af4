#!/bin/bash
# Round 6: the DP device path reduced in place (coalesced RCCL group per bucket, stats in place,
# status MAX): parity, step-time cost at C2 / C4 through a one-rank RCCL group (last bucket from the
# main stream vs the comm stream), and a kernel trace of the DP step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_r06i.log 2>&1 || { tail -30 gpurun_out/t_r06i.log; exit 1; }
tail -3 gpurun_out/t_r06i.log
for A in "" "--last-on-comm"; do
  timeout -k 10 300 python tools/dp_overhead.py $A > gpurun_out/dp_c2_i.json 2> gpurun_out/dp_c2_i.err || { tail -20 gpurun_out/dp_c2_i.err; exit 1; }
  cat gpurun_out/dp_c2_i.json
  timeout -k 10 400 python tools/dp_overhead.py $A --arch par/arch5.json --batch 32 --steps 8 > gpurun_out/dp_c4_i.json 2> gpurun_out/dp_c4_i.err || { tail -20 gpurun_out/dp_c4_i.err; exit 1; }
  cat gpurun_out/dp_c4_i.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_dp -o run -- python tools/dp_overhead.py --mode dp --rounds 1 --steps 14 > gpurun_out/prof_dp.log 2>&1 || exit 1
K=$(find gpurun_out/prof_dp -name '*kernel_trace.csv' | head -1)
python tools/step_timeline.py "$K" > gpurun_out/timeline_dp.txt 2>&1
echo r06i ok
