#!/bin/bash
# gpurun (round 4): the whole GPU suite + smoke on the FMA build, then the knob sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r04f"; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
grep -E "passed|failed|error" "$OUT/pytest_gpu.log" | tail -6
[ $rc -le 1 ] && timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; tail -1 "$OUT/smoke.log"
[ $rc -le 1 ] && TAG=r04f/sweep bash scripts/gpu_sweep_r04.sh
exit $rc
