#!/bin/bash
# gpurun: tiered-walk diagnosis — whole-frame A/B and a kernel trace of the tiered C2 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source scripts/gpu_step.sh
TAG=${TAG:-tier2}; OUT="$PWD/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp
step 300 "$OUT/diff_c2.log" python scripts/tier_diff.py random_spheres 1920 500 "$OUT/diff_c2.json"
tail -1 "$OUT/diff_c2.log"
step 300 "$OUT/prof.log" rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --steps 3 --warmup 1 --no-cpu --no-hash
cat "$OUT"/prof/*/run_kernel_stats.csv 2>/dev/null | cut -c1-200 | head -8
