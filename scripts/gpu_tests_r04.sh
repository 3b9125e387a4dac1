#!/bin/bash
# gpurun (round 4): the whole GPU suite and smoke on this library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-tests04}"; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1 && \
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?
grep -E "passed|failed|error" "$OUT/pytest_gpu.log" | tail -6; tail -2 "$OUT/smoke.log" 2>/dev/null
exit $rc
