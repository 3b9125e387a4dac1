#!/bin/bash
# gpurun (the final library of a round, part 1): PMC profiles of every bench workload (gpu_profiles.sh, copied into
# profiles/ on the box so the bench lines after it derive their roofline), the headline bench at the driver's 20
# steps, and the rocprofv3 kernel trace of the driver's bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${ROUND:-06}; OUT="$PWD/gpurun_out/final$R"; mkdir -p "$OUT"; export TMPDIR=/tmp
ROUND=$R bash scripts/gpu_profiles.sh > "$OUT/profiles.txt" 2>&1 || { tail -20 "$OUT/profiles.txt"; exit 1; }
tail -3 "$OUT/profiles.txt" | cut -c1-200
timeout -k 10 400 python bench.py --steps 20 --warmup 2 > "$OUT/bench_k20.json" 2> "$OUT/bench_k20.err" || { tail "$OUT/bench_k20.err"; exit 1; }
cut -c1-300 "$OUT/bench_k20.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o run --output-format csv -- \
    python bench.py --no-cpu > "$OUT/bench_under_rocprof.json" 2> "$OUT/bench_under_rocprof.err" || { tail "$OUT/bench_under_rocprof.err"; exit 1; }
cut -c1-200 "$OUT/bench_under_rocprof.json"
