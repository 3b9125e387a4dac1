#!/bin/bash
# gpurun: the GPU test suite (one process, per-test time limit) then smoke.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out"; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1 && \
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?
echo "exit=$rc"; grep -E "passed|failed|error" "$OUT/pytest_gpu.log" | tail -5; cat "$OUT/smoke.log" 2>/dev/null | tail -3
exit $rc
