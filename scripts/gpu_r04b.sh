#!/bin/bash
# gpurun (round 4): the tests that failed in r04a, then C2 with a 64-record queue (the redo pass's
# cost when nearly every deferred path overflows), C4 once more.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r04b"; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    -k "shard_run or kernel_variant or stress_100k or nested_world or watchdog or ties or walk_layout or go_sequence" > "$OUT/pytest_gpu.log" 2>&1
rc=$?
grep -E "passed|failed|error" "$OUT/pytest_gpu.log" | tail -8
[ $rc -le 1 ] && \
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu > "$OUT/c2.json" 2> "$OUT/c2.err" && tail -1 "$OUT/c2.json" && \
RTX_DEFER_CAP=64 timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu > "$OUT/c2_cap64.json" 2> "$OUT/c2_cap64.err" && tail -1 "$OUT/c2_cap64.json" && \
timeout -k 10 240 python bench.py --scene stress_100k --width 1920 --spp 100 --steps 3 --warmup 1 --no-cpu > "$OUT/c4.json" 2> "$OUT/c4.err" && tail -1 "$OUT/c4.json"
echo "rc=$rc $?"
