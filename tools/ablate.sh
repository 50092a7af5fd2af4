#!/bin/bash
# Build timing-only ablation variants of liblbwn.so (layer kernels) into lb-wavenet_amd/lbwn/abl/.
# Usage: bash tools/ablate.sh 0 1 2 4 ...
set -e
cd "$(dirname "$0")/../lb-wavenet_amd/csrc"
mkdir -p ../lbwn/abl build/abl
for A in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DLBWN_ABL=$A -c layer.hip -o build/abl/layer_$A.o
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC build/gemm.o build/abl/layer_$A.o build/misc.o build/gen.o build/cond.o build/engine.o build/capi.o -o ../lbwn/abl/liblbwn_abl$A.so
done
