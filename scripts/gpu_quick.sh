#!/bin/bash
# gpurun: quick parity gate (short limits) then an optional A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out"; mkdir -p "$OUT"; export TMPDIR=/tmp
export RTX_WATCHDOG_S=${RTX_WATCHDOG_S:-60}
timeout -k 10 ${TEST_LIMIT:-150} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest exit=$rc"; tail -15 "$OUT/pytest_gpu.log"
[ $rc -ne 0 ] && exit $rc
if [ -n "$AB_ARGS" ]; then
  timeout -k 10 ${AB_LIMIT:-400} python scripts/ab.py $AB_ARGS > "$OUT/ab.log" 2>&1; rc=$?
  echo "ab exit=$rc"; cat "$OUT/ab.log"
fi
exit $rc
