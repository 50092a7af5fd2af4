#!/bin/bash
# generation parity tests + same-box A/B against a variant build + the wall-clock trace.  Usage: VARIANT
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gen.py > gpurun_out/pytest_gen.log 2>&1 || { tail -30 gpurun_out/pytest_gen.log; exit 1; }
tail -2 gpurun_out/pytest_gen.log
bash tools/gen_ab.sh $1 > gpurun_out/gen_ab.txt 2>&1 || { cat gpurun_out/gen_ab.txt; exit 1; }
cat gpurun_out/gen_ab.txt
timeout -k 10 120 python tools/gen_trace.py 10 > gpurun_out/gen_trace_ab.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/gen_trace_ab.txt
