# The GPU test suite on the box, one process, per-test timeout; log under gpurun_out/.
# Usage: bash tools/gpu_tests.sh TAG [pytest -k expression]
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-t}
ARGS=(tests -m gpu -x -v --timeout 300 --timeout-method thread)
[ -n "$2" ] && ARGS+=(-k "$2")
timeout -k 10 900 python -u -m pytest "${ARGS[@]}" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_$TAG.log
exit $rc
