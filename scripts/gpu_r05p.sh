#!/bin/bash
# gpurun (round 5): C1 (400x225x100) kernel trace with timestamps — the near pass, far pass and their gaps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/${P_TAG:-r05p}"; mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c1" -o run --output-format csv -- \
    python bench.py --width 400 --spp 100 --steps 10 --warmup 1 --no-cpu > "$OUT/c1_prof.log" 2>&1 || { tail -20 "$OUT/c1_prof.log"; exit 1; }
tail -1 "$OUT/c1_prof.log" | cut -c1-200
