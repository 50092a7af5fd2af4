#!/bin/bash
# Round-6: chain traces (export form / in-chain) and the export-store placement A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
LBWN_BWD_WGRAD=1 timeout -k 10 120 python tools/chain_trace.py > gpurun_out/ct_wg1.txt 2>&1 || { tail -20 gpurun_out/ct_wg1.txt; exit 1; }
cat gpurun_out/ct_wg1.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "wg and (plan_forward_backward or conditioning or shorter or staged)" > gpurun_out/t_wg.log 2>&1 || { tail -40 gpurun_out/t_wg.log; exit 1; }
tail -2 gpurun_out/t_wg.log
LBWN_BWD_WGRAD=1 bash tools/ab_lib.sh wglate lb-wavenet_amd/lbwn/abl/liblbwn_gearly.so || exit 1
echo wg2 ok
