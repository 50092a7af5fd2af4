#!/bin/bash
# Session-3 GPU pass: the full-size parity tests, then the HBM traffic PMC passes at HEAD.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "fullsize or full_size or restatement or adam" -x -v --timeout 300 --timeout-method thread > gpurun_out/t_full.log 2>&1 || { echo "fullsize tests failed"; tail -40 gpurun_out/t_full.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/t_full.log | tail -5
bash tools/pmc_traffic.sh > gpurun_out/pmc.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc.log; exit 1; }
cp gpurun_out/pmc_traffic/pmc_traffic.json gpurun_out/pmc_traffic_head.json
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --no-gen --steps 30 > gpurun_out/b_quick.json 2> gpurun_out/b_quick.err || { echo "bench failed"; tail -5 gpurun_out/b_quick.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/b_quick.json')); print('C2', d['ms_per_step'], 'bwd', d['roofline']['avg_launch_us'], 'fwd', d['roofline_dilconv']['avg_launch_us'])"
echo "r3s3 ok"
