#!/bin/bash
# gpurun (round 4, final library): the driver's default bench command, a rocprofv3 kernel trace of the
# same command (profiles/r04_kernel_stats.csv), then one bench line per config (gpu_configs_r04.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/final04"; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && tail -1 "$OUT/bench.json" | cut -c1-300 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --no-cpu > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" && \
TAG=final04/configs bash scripts/gpu_configs_r04.sh
rc=$?
echo "final rc=$rc"
exit $rc
