#!/bin/bash
# gpurun (round 5, final library): C2 knobs around the defaults once more (shade threshold, miss-phase hits, primitive
# batch, samples per unit), alternating in one process.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r05ah"; mkdir -p "$OUT"
timeout -k 10 600 python scripts/ab.py --spp 500 --rounds 2 \
    --variants "v3,v3@RTX_SHADE_THRESH=50,v3@RTX_SHADE_THRESH=54,v3@RTX_REFILL_HITS=32,v3@RTX_REFILL_HITS=40,v3@RTX_PRIM_BATCH=10,v3@RTX_PRIM_BATCH=14,v3@RTX_ITEM_SUB=32" \
    > "$OUT/c2.log" 2>&1 || { tail -5 "$OUT/c2.log"; exit 1; }
grep -h "sha256\|median" "$OUT/c2.log"
