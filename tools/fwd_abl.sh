#!/bin/bash
# Forward-chain store ablations (timing only, tools/ablate.sh variants): chain trace + layer_fwd time
# per variant.  Usage (on the box): bash tools/fwd_abl.sh A1 A2 ...
set -o pipefail
mkdir -p gpurun_out
for A in "$@"; do
  export LBWN_LIB=lb-wavenet_amd/lbwn/abl/liblbwn_abl$A.so
  echo "== LBWN_ABL=$A"
  timeout -k 10 120 python tools/chain_trace.py 1 > gpurun_out/fabl_$A.txt 2>&1 || { echo "trace $A failed"; tail gpurun_out/fabl_$A.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/fabl_$A.txt | sed -n '1,12p'
done
