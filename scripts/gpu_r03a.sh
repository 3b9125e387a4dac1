#!/bin/bash
# gpurun: the whole GPU suite (no -x: every failure listed), smoke, then the headline bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-r03a}"; mkdir -p "$OUT"; export TMPDIR=/tmp
export RTX_WATCHDOG_S=${RTX_WATCHDOG_S:-120}
timeout -k 10 ${TEST_LIMIT:-700} python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
    ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest exit=$rc"; grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest_gpu.log" | tail -25
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
tail -2 "$OUT/smoke.log"
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
tail -1 "$OUT/bench.json"
exit $rc
