#!/bin/bash
# gpurun (round 5): config 4's kernel trace (near / far / redo / reduce per step).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r05z"; mkdir -p "$OUT"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python bench.py --scene stress_100k --spp 100 --no-cpu --steps 3 --warmup 1 > "$OUT/c4.json" 2> "$OUT/trace.log" || { tail -5 "$OUT/trace.log"; exit 1; }
find "$OUT/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
cut -d, -f1-4 "$OUT/kernel_stats.csv" | head -8
