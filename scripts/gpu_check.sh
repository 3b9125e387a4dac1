#!/bin/bash
# One gpurun call: GPU parity tests, smoke, bench, and a rocprofv3 kernel-trace profile
# of the bench.  Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS="${STEPS:-3}"
timeout -k 10 400 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && \
timeout -k 10 400 python bench.py --steps "$STEPS" --warmup 1 --cpu-target-s 10 > "$OUT/bench.log" 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --steps 2 --warmup 1 --no-cpu > "$OUT/bench_prof.log" 2>&1
rc=$?
echo "exit=$rc"
tail -3 "$OUT/pytest_gpu.log"; cat "$OUT/smoke.log" 2>/dev/null; tail -2 "$OUT/bench.log" 2>/dev/null
exit $rc
