#!/bin/bash
# SQ counter passes (counters only, one pass per group) over a command (default: tools/gemm_bench.py
# for the shapes in $GEMM_ONLY; PMC_CMD overrides, e.g. "python bench.py --steps 4 --no-gen
# --no-cpu-baseline"), averaged per kernel whose name contains $PMC_KERNELS (comma list).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_gemm
mkdir -p $OUT
CMD=${PMC_CMD:-python tools/gemm_bench.py}
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM_RD" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $C --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $OUT/p$i.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections, os
keys = os.environ.get('PMC_KERNELS', 'gemm_f32,gemm_x3').split(',')
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob('gpurun_out/pmc_gemm/p*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if any(k in r['Kernel_Name'] for k in keys):
            agg[r['Kernel_Name'].replace('(anonymous namespace)::', '')[:70]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print('   %-28s %14.0f  (n=%d)' % (c, sum(v) / len(v), len(v)))
PY
