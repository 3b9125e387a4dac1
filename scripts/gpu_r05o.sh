#!/bin/bash
# gpurun (round 5): parked lanes off the sentinel's HBM read in the walk of a scene in HBM (RTX_HYB_SENTINEL) —
# config 4 A/B against the build without it (abl/librtx_nosent.so), alternating; then the stress-scene parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r05o"; mkdir -p "$OUT"
for i in 1 2; do
  for lib in cur nosent; do
    L=""; [ $lib != cur ] && L="RTX_LIB=$PWD/abl/librtx_$lib.so"
    timeout -k 10 240 env $L python scripts/ab.py --scene stress_100k --spp 100 --rounds 2 --variants v3 > "$OUT/c4_${lib}_$i.log" 2>&1 || { tail -5 "$OUT/c4_${lib}_$i.log"; exit 1; }
    echo "$lib $(grep median "$OUT/c4_${lib}_$i.log" | head -1)"
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "stress or C4" > "$OUT/pytest.log" 2>&1 || { tail -20 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
