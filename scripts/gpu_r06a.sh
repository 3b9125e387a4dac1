#!/bin/bash
# round 6: the sticky error word's tests, then the headline bench at the driver's 20 steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r06a"; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_claim_guard.py -x -v --timeout 300 --timeout-method thread \
    > "$OUT/claim.log" 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
echo "exit=$rc"; tail -3 "$OUT/claim.log"; cat "$OUT/bench.json"
exit $rc
