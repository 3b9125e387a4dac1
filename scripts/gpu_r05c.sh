#!/bin/bash
# gpurun (round 5): guard v2 (uniform flag), camera-ray pool for tiered and untiered LDS scenes, miss phases
# (RTX_REFILL_HITS).  The whole GPU suite with miss phases on (every LDS render takes them), then A/Bs in one
# process per build: C2 (1920x1080x500) and the Cornell box (600x600x200).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-r05c}"; mkdir -p "$OUT"; export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
RTX_REFILL_HITS=40 timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
grep -E "passed|failed|error" "$OUT/pytest_gpu.log" | tail -4
[ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" "$OUT/pytest_gpu.log" | head -80; exit $rc; }
fi
V="v3,v3@RTX_REFILL_HITS=32,v3@RTX_REFILL_HITS=40,v3@RTX_REFILL_HITS=48,v3@RTX_CAM_POOL=0"
for i in 1 2; do
  timeout -k 10 200 python scripts/ab.py --spp 500 --rounds 3 --variants $V > "$OUT/ab_c2_$i.log" 2>&1 || exit 1
  grep "median\|sha256" "$OUT/ab_c2_$i.log" | head -6
  RTX_LIB=$PWD/abl/librtx_r04.so timeout -k 10 200 python scripts/ab.py --spp 500 --rounds 3 --variants v3 > "$OUT/ab_r04_$i.log" 2>&1 || exit 1
  echo "r04  $(grep "median" "$OUT/ab_r04_$i.log" | head -1)"
done
timeout -k 10 200 python scripts/ab.py --scene cornell_box --width 600 --spp 200 --rounds 3 --variants $V > "$OUT/ab_cornell.log" 2>&1 || exit 1
grep "median\|sha256" "$OUT/ab_cornell.log" | head -6
RTX_LIB=$PWD/abl/librtx_r04.so timeout -k 10 200 python scripts/ab.py --scene cornell_box --width 600 --spp 200 --rounds 3 --variants v3 > "$OUT/ab_cornell_r04.log" 2>&1 || exit 1
echo "r04  $(grep "median" "$OUT/ab_cornell_r04.log" | head -1)"
