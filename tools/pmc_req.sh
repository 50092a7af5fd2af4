#!/bin/bash
# HBM read requests by size per launch (MI355X_MICROARCH.md § HBM: FETCH_SIZE = 128·BUBBLE +
# 64·(RDREQ - BUBBLE - RDREQ_32B) + 32·RDREQ_32B; on gfx950 wide streaming reads come out at ½):
# one counter-only pass with the three TCC request counters, mapped to bench probe names.
# Usage (on the GPU box): bash tools/pmc_req.sh [bench args...]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_req
mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum --output-format csv -d $OUT/req -o run -- \
    python bench.py --steps 4 --warmup 8 --no-gen --no-cpu-baseline --no-extras "$@" > $OUT/req.log 2>&1 || { echo "req pass failed"; tail -5 $OUT/req.log; exit 1; }
python tools/pmc_req.py $OUT/req $OUT/pmc_req.json
