#!/bin/bash
# MFMA-busy counters per launch (one counter-only pass, no tracing domains) for the training step
# of one configuration or for generation.  Usage (GPU box):
#   TAG=c2 bash tools/pmc_mfma.sh train [bench args...]     e.g. --arch par/arch5.json --batch 32
#   TAG=gen bash tools/pmc_mfma.sh gen  [gen_bench args...]
set -o pipefail
export TMPDIR=/tmp
MODE=$1; shift
OUT=gpurun_out/pmc_mfma_${TAG:-x}
mkdir -p $OUT
C="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
if [ "$MODE" = gen ]; then
  CMD="python tools/gen_bench.py --batch 10 --steps 600 $*"
else
  CMD="python bench.py --steps 4 --warmup 6 --no-gen --no-cpu-baseline --no-extras $*"
fi
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $OUT/p -o run -- $CMD > $OUT/run.log 2>&1 || { echo "pmc pass failed"; tail -5 $OUT/run.log; exit 1; }
python tools/pmc_mfma.py $OUT/p $OUT/pmc_mfma_${TAG:-x}.json "$MODE $*"
