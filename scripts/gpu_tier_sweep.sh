#!/bin/bash
# gpurun: tier tests + bench A/B (gpu_tier.sh), then the knob sweep (scripts/sweep.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_tier.sh || exit $?
source scripts/gpu_step.sh
OUT="$PWD/gpurun_out/${TAG:-tier}"
step 400 "$OUT/sweep.jsonl" python scripts/sweep.py --thresh ${THRESH:-40,44,48,52,56} --batch ${BATCH:-12,16,20} --tier 1
cat "$OUT/sweep.jsonl" | grep '"tier"' | cut -c1-80
