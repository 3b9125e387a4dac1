#!/bin/bash
# gpurun (round 4): where a rank's time goes at N = 8 (rank 0's rows alone, rocprof kernel trace).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r04g"; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_s8" -o run --output-format csv -- python bench.py --shard 0/8 --steps 5 --warmup 1 --no-cpu > "$OUT/s8.json" 2> "$OUT/s8.err" && tail -1 "$OUT/s8.json" | cut -c1-200
