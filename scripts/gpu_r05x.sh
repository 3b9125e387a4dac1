#!/bin/bash
# gpurun (round 5): with the drain, C1's unit size and grid (RTX_ITEM_SUB, RTX_ITEM_GRID) around the automatic choice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r05x"; mkdir -p "$OUT"
timeout -k 10 300 python scripts/ab.py --width 400 --spp 100 --rounds 5 \
    --variants "v3,v3@RTX_ITEM_SUB=1,v3@RTX_ITEM_SUB=4,v3@RTX_ITEM_GRID=75,v3@RTX_ITEM_GRID=50,v3@RTX_DRAIN=0" > "$OUT/c1.log" 2>&1 || { tail -5 "$OUT/c1.log"; exit 1; }
grep -h "sha256\|median" "$OUT/c1.log"
