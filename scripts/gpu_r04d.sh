#!/bin/bash
# gpurun (round 4): where the time goes when the queue overflows (rocprof kernel stats at RTX_DEFER_CAP=64
# and at the default), the Go-sequence tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r04d"; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "go_sequence or overflow or ties or stress_100k_crop" > "$OUT/pytest_gpu.log" 2>&1
rc=$?
grep -E "passed|failed|error" "$OUT/pytest_gpu.log" | tail -4
[ $rc -le 1 ] && \
RTX_DEFER_CAP=64 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_cap64" -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu > "$OUT/c2_cap64.json" 2> "$OUT/c2_cap64.err" && tail -1 "$OUT/c2_cap64.json" | cut -c1-200 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2" -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu > "$OUT/c2.json" 2> "$OUT/c2.err" && tail -1 "$OUT/c2.json" | cut -c1-200
echo "rc=$rc $?"
