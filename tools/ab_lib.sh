#!/bin/bash
# Same-box A/B of library builds on the training step: the default in-tree build against one or
# more variants (tools/build_variant.sh), interleaved over two rounds; prints ms_per_step and the
# probed dominant-kernel / forward-chain launch times per arm.  Optional bench args after "--".
# Usage: bash tools/ab_lib.sh TAG VARIANT.so [VARIANT2.so ...] [-- bench args]
set -o pipefail
TAG=$1; shift
ARMS=(default); BARGS=()
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; BARGS=("$@"); break; fi
  ARMS+=("$1"); shift
done
mkdir -p gpurun_out
for round in 1 2; do
  i=0
  for A in "${ARMS[@]}"; do
    i=$((i + 1))
    O=gpurun_out/ab_${TAG}_${i}_$round.json
    if [ "$A" = default ]; then
      timeout -k 10 150 python bench.py --no-cpu-baseline --no-extras --no-gen "${BARGS[@]}" > $O 2> $O.err || { echo "arm $i failed"; tail -5 $O.err; exit 1; }
    else
      timeout -k 10 150 python tools/with_lib.py "$A" bench.py --no-cpu-baseline --no-extras --no-gen "${BARGS[@]}" > $O 2> $O.err || { echo "arm $i ($A) failed"; tail -5 $O.err; exit 1; }
    fi
    python - "$O" "$round" "$i" "$A" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r, rd = d['roofline'], d['roofline_dilconv']
print('round %s arm%s %-40s %.4f ms/step  %s %.1f us  layer_fwd %.1f us' % (
    sys.argv[2], sys.argv[3], sys.argv[4][-40:], d['ms_per_step'], r['kernel'], r['avg_launch_us'], rd['avg_launch_us']))
PY
  done
done
echo ab ok
