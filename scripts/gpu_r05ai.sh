#!/bin/bash
# gpurun (round 5, final library): walk steps between two wave votes (RTX_WALK_STEPS 4 / 6 / 8) on C2, alternating builds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r05ai"; mkdir -p "$OUT"
for i in 1 2; do
  for lib in cur steps4 steps8; do
    L=""; [ $lib != cur ] && L="RTX_LIB=$PWD/abl/librtx_$lib.so"
    timeout -k 10 240 env $L python scripts/ab.py --spp 500 --rounds 2 --variants v3 > "$OUT/c2_${lib}_$i.log" 2>&1 || { tail -5 "$OUT/c2_${lib}_$i.log"; exit 1; }
    echo "$lib $(grep -h 'sha256\|median' "$OUT/c2_${lib}_$i.log" | tr '\n' ' ' | cut -c1-160)"
  done
done
