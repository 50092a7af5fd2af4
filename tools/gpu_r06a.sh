#!/bin/bash
# Round 6: full GPU suite + C4 / C2 bench after the side-stream GC kernels.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_tests.sh r06a || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r06a.log 2>&1 || { tail -5 gpurun_out/smoke_r06a.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r06a.json 2> gpurun_out/bench_r06a.err || { tail -20 gpurun_out/bench_r06a.err; exit 1; }
echo r06a ok
