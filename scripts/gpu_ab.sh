#!/bin/bash
# gpurun: GPU parity tests, then an interleaved A/B of kernel variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out"; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 && \
timeout -k 10 600 python scripts/ab.py ${AB_ARGS:---spp 100 --rounds 3 --variants v3,nolds} > "$OUT/ab.log" 2>&1
rc=$?
echo "exit=$rc"; tail -3 "$OUT/pytest_gpu.log"; cat "$OUT/ab.log"
exit $rc
