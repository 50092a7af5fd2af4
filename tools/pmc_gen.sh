#!/bin/bash
# PMC passes (counters only, one group per run, no tracing domains) over the persistent
# generation kernel (tools/gen_bench.py, arch3, B=10), then a per-kernel summary.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_gen
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_gen/p$i -o run -- python tools/gen_bench.py --batch 10 --steps 400 --chunk 100 > gpurun_out/pmc_gen/p$i.log 2>&1 || echo "pass $i failed"
done
python tools/pmc_summary.py gpurun_out/pmc_gen gen_persist > gpurun_out/pmc_gen/summary.txt
echo done
