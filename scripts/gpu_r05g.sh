#!/bin/bash
# gpurun (round 5): the measurement set of the round-5 library — PMC profiles of every bench workload
# (scripts/gpu_profiles_r05.sh), the kernel trace of the driver's default bench command, and every rank's shard.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/${TRACE_TAG:-r05g}"; mkdir -p "$OUT"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python bench.py --no-cpu \
    > "$OUT/bench_under_rocprof.json" 2> "$OUT/trace.log" || { tail -5 "$OUT/trace.log"; exit 1; }
find "$OUT/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
head -6 "$OUT/kernel_stats.csv" | cut -c1-220
TAG=prof05 bash scripts/gpu_profiles_r05.sh || exit 1
TAG=shards05 bash scripts/gpu_shards_r05.sh || exit 1
