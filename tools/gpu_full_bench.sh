#!/bin/bash
# GPU tests, then the full bench line (all sub-objects).  Usage: bash tools/gpu_full_bench.sh TAG
set -o pipefail
TAG=$1
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -rA > gpurun_out/t_$TAG.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_$TAG.log; exit 1; }
grep -E "passed|failed|train.py .* ms/step" gpurun_out/t_$TAG.log | tail -3
timeout -k 10 600 python bench.py > gpurun_out/bench_full_$TAG.json 2> gpurun_out/bench_full_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_full_$TAG.err; exit 1; }
python - <<PY
import json; d=json.load(open('gpurun_out/bench_full_$TAG.json'))
print('C2', d['ms_per_step'], d['value'], 'bwd', d['roofline']['avg_launch_us'], 'fwd', d['roofline_dilconv']['avg_launch_us'])
for k in ['c4','c5_per_gpu','c1']: print(k, d[k]['ms_per_step'])
g=d['gen']; print('gen', g['us_per_step'], [(s['batch'], round(s['us_per_step'],1), s['form']) for s in g['sweep']])
print([ (r['d'], r['fwd_cycles'], r['bwd_cycles']) for r in d['c4']['sweep']['per_dilation']])
PY
echo "full $TAG ok"
