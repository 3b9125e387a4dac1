#!/bin/bash
# gpurun (round 5, first call): the new tests (claim guard, PPM on device 0 for any band count), the whole
# GPU suite and smoke, then the guarded library against round 4's (abl/librtx_r04.so) on C2 (1920x1080x500).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-r05a}"; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_claim_guard.py tests/test_ppm_gpu.py tests/test_go_binding.py -m gpu -x -v \
    --timeout 200 --timeout-method thread > "$OUT/pytest_new.log" 2>&1 || { tail -30 "$OUT/pytest_new.log"; exit 1; }
grep -E "passed|failed" "$OUT/pytest_new.log" | tail -2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 && \
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?
grep -E "passed|failed|error" "$OUT/pytest_gpu.log" | tail -4; tail -2 "$OUT/smoke.log" 2>/dev/null
[ $rc -eq 0 ] || exit $rc
ARGS="--spp 500 --rounds 3 --variants v3"
for i in 1 2; do
  timeout -k 10 200 python scripts/ab.py $ARGS > "$OUT/ab_cur_$i.log" 2>&1 || exit 1
  echo "cur  $(grep "median\|sha256" "$OUT/ab_cur_$i.log" | head -3 | tr '\n' ' ')"
  RTX_LIB=$PWD/abl/librtx_r04.so timeout -k 10 200 python scripts/ab.py $ARGS > "$OUT/ab_r04_$i.log" 2>&1 || exit 1
  echo "r04  $(grep "median\|sha256" "$OUT/ab_r04_$i.log" | head -3 | tr '\n' ' ')"
done
