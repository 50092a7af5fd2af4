#!/bin/bash
# Same-box A/B: per-wave forward hand-offs vs the per-tile flag protocol (variant build from the
# commit before), the XCD-grouped chain tile walk, and dZ's 2-D XCD blocking.
set -o pipefail
mkdir -p gpurun_out
V=lb-wavenet_amd/lbwn/abl/liblbwn_gtileflag.so
CONFIGS="arch3:8 arch5:8" bash tools/ab_env.sh "-" "LBWN_CHAIN_XCD=0" "LBWN_LIB=$V" "LBWN_LIB=$V LBWN_CHAIN_XCD=0" "LBWN_DZ_XCD=0" > gpurun_out/ab3.txt 2>&1 || { cat gpurun_out/ab3.txt; exit 1; }
cat gpurun_out/ab3.txt
