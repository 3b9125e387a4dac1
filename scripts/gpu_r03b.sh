#!/bin/bash
# gpurun: tree variants on the headline (bench lines), then the GPU suite without -x and smoke.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03b} VARIANTS="${VARIANTS:-RTX_BVH=guarded;RTX_BVH=sah;RTX_BVH=reference}" \
    BENCH_ARGS="${BENCH_ARGS:---steps 5 --warmup 1}" bash scripts/gpu_variants.sh || exit $?
OUT="$PWD/gpurun_out/${TAG:-r03b}"; export TMPDIR=/tmp RTX_WATCHDOG_S=120
timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
    ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest exit=$rc"; grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest_gpu.log" | tail -25
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
tail -1 "$OUT/smoke.log"
exit $rc
