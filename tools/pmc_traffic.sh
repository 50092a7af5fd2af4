#!/bin/bash
# HBM traffic per launch (MI355X_MICROARCH.md § HBM): FETCH_SIZE and WRITE_SIZE in SEPARATE
# counter-only passes (no tracing domains) over a short bench run, then tools/pmc_traffic.py
# maps dispatches to bench probe names and applies the gfx950 FETCH_SIZE x2 correction.
# Usage (on the GPU box): [TAG=c4] bash tools/pmc_traffic.sh [bench args...]
# (TAG names the output: gpurun_out/pmc_traffic[_TAG]/pmc_traffic[_TAG].json; LIB=<variant .so>
# profiles a same-box A/B variant build through tools/with_lib.py)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_traffic${TAG:+_$TAG}
mkdir -p $OUT
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $C --output-format csv -d $OUT/$C -o run -- \
      python ${LIB:+tools/with_lib.py $LIB} bench.py --steps 4 --warmup 8 --no-gen --no-cpu-baseline --no-extras "$@" > $OUT/$C.log 2>&1 || { echo "pass $C failed"; tail -5 $OUT/$C.log; exit 1; }
done
python tools/pmc_traffic.py $OUT/FETCH_SIZE $OUT/WRITE_SIZE $OUT/pmc_traffic${TAG:+_$TAG}.json
