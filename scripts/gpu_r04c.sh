#!/bin/bash
# gpurun (round 4): the redo pass from a compacted list — overflow tests, then C2 at RTX_DEFER_CAP=64 / 1e5 / default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r04c"; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    -k "overflow or shard_run or kernel_variant or stress_100k or nested_world or watchdog or ties or go_sequence" > "$OUT/pytest_gpu.log" 2>&1
rc=$?
grep -E "passed|failed|error" "$OUT/pytest_gpu.log" | tail -8
[ $rc -le 1 ] && \
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu > "$OUT/c2.json" 2> "$OUT/c2.err" && tail -1 "$OUT/c2.json" | cut -c1-300 && \
RTX_DEFER_CAP=64 timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu > "$OUT/c2_cap64.json" 2> "$OUT/c2_cap64.err" && tail -1 "$OUT/c2_cap64.json" | cut -c1-300 && \
RTX_DEFER_CAP=100000 timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu > "$OUT/c2_cap1e5.json" 2> "$OUT/c2_cap1e5.err" && tail -1 "$OUT/c2_cap1e5.json" | cut -c1-300
echo "rc=$rc $?"
