#!/bin/bash
# gpurun (round 5): the reduction with 8 colours in flight per thread: its kernel time (trace of the default bench) and
# the parity tests that read its output (every GPU frame test goes through it).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r05af"; mkdir -p "$OUT"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python bench.py --no-cpu \
    > "$OUT/bench_under_rocprof.json" 2> "$OUT/trace.log" || { tail -5 "$OUT/trace.log"; exit 1; }
find "$OUT/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
cut -d, -f1-4 "$OUT/kernel_stats.csv" | grep -E "reduce|drain"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "config1 or chunked or drain or overflow" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
