#!/bin/bash
# Session-3 pass 2: the whole -m gpu suite at HEAD, the generation variants' draws (gen tests under
# each variant library) and same-box A/B, then the full measurement pass (bench line, profiles).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
for v in sk skrw; do
  LBWN_LIB=lb-wavenet_amd/lbwn/abl/liblbwn_g$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_gen.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gen_$v.log 2>&1 && echo "gen tests $v: $(tail -1 gpurun_out/t_gen_$v.log)" || echo "gen tests $v FAILED: $(grep -E 'differ|assert' gpurun_out/t_gen_$v.log | head -3)"
done
bash tools/gen_ab.sh rw sk skrw || exit 1
bash tools/gpu_full.sh r03_v4 || exit 1
echo "r3s3b ok"
