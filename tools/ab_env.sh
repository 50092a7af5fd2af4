#!/bin/bash
# Same-box A/B of plan switches on the training step: each arm is an env assignment list
# ("" = defaults), interleaved over two rounds; prints ms_per_step and the probed dominant-kernel /
# forward-chain launch times per arm.  Optional bench args after "--".
# Usage: bash tools/ab_env.sh TAG "A=1 B=2" "A=0" [-- bench args]
set -o pipefail
TAG=$1; shift
ARMS=(); BARGS=()
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; BARGS=("$@"); break; fi
  ARMS+=("$1"); shift
done
mkdir -p gpurun_out
for round in 1 2; do
  i=0
  for A in "${ARMS[@]}"; do
    i=$((i + 1))
    O=gpurun_out/abe_${TAG}_${i}_$round.json
    env $A timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --no-gen "${BARGS[@]}" > $O 2> $O.err || { echo "arm $i ($A) failed"; tail -5 $O.err; exit 1; }
    python - "$O" "$round" "$i" "$A" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r, rd = d['roofline'], d['roofline_dilconv']
w = d.get('warmup_probe_ms', {})
print('round %s arm%s %-32s %.4f ms/step  %s %.1f us  layer_fwd %.1f us  warm %s' % (
    sys.argv[2], sys.argv[3], sys.argv[4][-32:], d['ms_per_step'], r['kernel'], r['avg_launch_us'], rd['avg_launch_us'],
    ' '.join('%s=%.0f' % (k, v * 1e3) for k, v in sorted(w.items()))))
PY
  done
done
echo ab ok
