#!/bin/bash
# gpurun (round 5): the camera-ray pool (render_items<POOL>) — the whole GPU suite, then C2 (1920x1080x500)
# A/B in one process per build: the pool, the pool off (RTX_CAM_POOL=0), round 4's library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-r05b}"; mkdir -p "$OUT"; export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
grep -E "passed|failed|error" "$OUT/pytest_gpu.log" | tail -4
[ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" "$OUT/pytest_gpu.log" | head -80; exit $rc; }
fi
ARGS="--spp 500 --rounds 3 --variants v3,v3@RTX_CAM_POOL=0"
for i in 1 2; do
  timeout -k 10 200 python scripts/ab.py $ARGS > "$OUT/ab_cur_$i.log" 2>&1 || exit 1
  echo "cur  $(grep "median\|sha256" "$OUT/ab_cur_$i.log" | head -3 | tr '\n' ' ')"
  RTX_LIB=$PWD/abl/librtx_r04.so timeout -k 10 200 python scripts/ab.py --spp 500 --rounds 3 --variants v3 > "$OUT/ab_r04_$i.log" 2>&1 || exit 1
  echo "r04  $(grep "median\|sha256" "$OUT/ab_r04_$i.log" | head -2 | tr '\n' ' ')"
done
