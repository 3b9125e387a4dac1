#!/bin/bash
# gpurun (round 5): the tiered chunk at the 32-bit id limit (tests/test_gpu_parity.py::test_tier_chunk_at_id_limit).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r05ab"; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "id_limit or drain" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
grep -E "PASSED|FAILED|passed|failed" "$OUT/pytest.log" | tail -8
