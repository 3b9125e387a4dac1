#!/bin/bash
# gpurun (round 4, first pass): C4 and C2 bench lines on the new build, then the GPU suite (no -x:
# every failure listed), then smoke.  Every GPU step under its own time limit, chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r04a"; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 240 python bench.py --scene stress_100k --width 1920 --spp 100 --steps 2 --warmup 1 --no-cpu > "$OUT/c4.json" 2> "$OUT/c4.err" && \
tail -1 "$OUT/c4.json" && \
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu > "$OUT/c2.json" 2> "$OUT/c2.err" && \
tail -1 "$OUT/c2.json" && \
timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
grep -E "passed|failed|error" "$OUT/pytest_gpu.log" | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] && timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "pytest rc=$rc smoke rc=$?"; tail -3 "$OUT/smoke.log"
exit $rc
