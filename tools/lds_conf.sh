#!/bin/bash
# LDS bank-conflict attribution for chain_bwd_x3_kernel.
#   CPU side (this container):  bash tools/lds_conf.sh build     -> lb-wavenet_amd/lbwn/conf/liblbwn_confN.so
#   GPU side (on the box):      bash tools/lds_conf.sh run       -> gpurun_out/conf/summary.txt
# Each variant sends one group of the kernel's LDS accesses to a conflict-free address
# (layer.hip LBWN_CONF); SQ_LDS_BANK_CONFLICT of the kernel per variant, against the real build (0).
set -o pipefail
BITS="${CONF_BITS:-0 1024 2048 256 4095 5119}"
if [ "$1" = build ]; then
  cd "$(dirname "$0")/../lb-wavenet_amd/csrc"
  mkdir -p ../lbwn/conf build/conf
  for A in $BITS; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DLBWN_CONF=$A -c layer.hip -o build/conf/layer_$A.o || exit 1
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC build/gemm.o build/conf/layer_$A.o build/misc.o build/gen.o \
        build/cond.o build/engine.o build/capi.o -o ../lbwn/conf/liblbwn_conf$A.so || exit 1
  done
  exit 0
fi
export TMPDIR=/tmp
OUT=gpurun_out/conf
mkdir -p $OUT
for A in $BITS; do
  LBWN_LIB=lb-wavenet_amd/lbwn/conf/liblbwn_conf$A.so timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS \
      --output-format csv -d $OUT/c$A -o run -- python tools/kbench.py --iters 2 --probes layer_bwd@25 > $OUT/c$A.log 2>&1 || { echo "variant $A failed"; tail -5 $OUT/c$A.log; exit 1; }
  echo "== LBWN_CONF=$A" >> $OUT/summary.txt
  python tools/pmc_summary.py $OUT/c$A chain_bwd_x3 >> $OUT/summary.txt
done
cat $OUT/summary.txt
