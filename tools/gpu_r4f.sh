#!/bin/bash
# round-4 A/B batch: generation head (MFMA) parity + A/B + trace, backward bias sums (DPP) A/B,
# dZ 160-column tiles A/B, with the parity tests that cover them
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_tests.sh r4f "gen or full_size or plan_forward_backward" || exit 1
bash tools/gen_ab.sh r3gen > gpurun_out/gen_ab_r4f.txt 2>&1; cat gpurun_out/gen_ab_r4f.txt
timeout -k 10 120 python tools/gen_trace.py 10 > gpurun_out/gentrace_r4f.txt 2>&1; cat gpurun_out/gentrace_r4f.txt
CONFIGS="arch3:8 arch5:8" timeout -k 10 700 bash tools/ab_step.sh r4bias prevdz > gpurun_out/ab_bias_r4f.txt 2>&1; cat gpurun_out/ab_bias_r4f.txt
for r in 1 2; do for w in 1 0; do
  LBWN_GEMM_WIDE=$w timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --no-gen --steps 30 > gpurun_out/abw_$w.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/abw_$w.json')); print('round $r wide $w', round(d['ms_per_step'],4))"
done; done
bash tools/gpu_tests.sh r4f_gran "gran" || exit 1
for r in 1 2; do for hv in flag:flag gran:flag gran:gran; do
  LBWN_FWD_HANDOFF=${hv%%:*} LBWN_BWD_HANDOFF=${hv#*:} timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --no-gen --steps 30 > gpurun_out/abh_$hv.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/abh_$hv.json')); print('round $r handoff $hv', round(d['ms_per_step'],4), 'fwd', round(d['roofline_dilconv']['avg_launch_us'],1), 'bwd', round(d['roofline']['avg_launch_us'],1))"
done; done
LBWN_FWD_HANDOFF=gran LBWN_BWD_HANDOFF=gran timeout -k 10 120 python tools/chain_trace.py > gpurun_out/chaintrace_gran.txt 2>&1; cat gpurun_out/chaintrace_gran.txt
