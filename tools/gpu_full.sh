# One full GPU measurement pass: tests-free cycle (bench + rocprof), the full bench line, the
# generation kernel stats / trace and its PMC passes.  Usage (on the box): bash tools/gpu_full.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-v2}
TESTS=${TESTS:-0} bash tools/gpu_cycle.sh $TAG || exit 1
timeout -k 10 500 python bench.py > gpurun_out/bench_full_$TAG.json 2> gpurun_out/bench_full_$TAG.err || { tail -20 gpurun_out/bench_full_$TAG.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gen_$TAG -o run -- python tools/gen_bench.py --batch 10 --steps 4000 > gpurun_out/prof_gen_$TAG.log 2>&1 || exit 1
S=$(find gpurun_out/prof_gen_$TAG -name '*kernel_stats.csv' | head -1)
python tools/prof_summary.py "$S" gpurun_out/stats_gen_$TAG.md 10 gen_$TAG
timeout -k 10 120 python tools/gen_trace.py 10 > gpurun_out/gentrace_$TAG.txt 2>&1
bash tools/pmc_gen.sh
echo final ok
