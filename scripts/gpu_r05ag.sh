#!/bin/bash
# gpurun (round 5): the redo bits across sample chunks (tests/test_gpu_parity.py::test_tier_overflow_across_chunks).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r05ag"; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "across_chunks or overflow_redo" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
grep -E "PASSED|FAILED|passed|failed" "$OUT/pytest.log" | tail -9
