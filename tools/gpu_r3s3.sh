#!/bin/bash
# Session-3 GPU pass: full-size parity, Adam, generation (grouped persistent form) tests, the gen
# batch sweep, the HBM traffic PMC passes at HEAD, quick C2 bench, C4 / C2 kernel profiles.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_gen.py -k "full_size or restatement or adam or gen" -x -v --timeout 300 --timeout-method thread > gpurun_out/t_full.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_full.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_full.log | tail -3
for b in 16 32 64 80; do
  timeout -k 10 120 python tools/gen_bench.py --batch $b --steps 2000 > gpurun_out/genb_$b.txt 2>&1 || { echo "gen bench $b failed"; tail -5 gpurun_out/genb_$b.txt; exit 1; }
  echo "B=$b $(tail -1 gpurun_out/genb_$b.txt)"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --no-gen --steps 30 > gpurun_out/b_quick.json 2> gpurun_out/b_quick.err || { echo "bench failed"; tail -5 gpurun_out/b_quick.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/b_quick.json')); print('C2', d['ms_per_step'], 'bwd', d['roofline']['avg_launch_us'], 'fwd', d['roofline_dilconv']['avg_launch_us'])"
bash tools/pmc_traffic.sh > gpurun_out/pmc.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc.log; exit 1; }
cp gpurun_out/pmc_traffic/pmc_traffic.json gpurun_out/pmc_traffic_head.json
bash tools/prof_arch.sh c4 par/arch5.json --batch 32 || exit 1
echo "r3s3 ok"
