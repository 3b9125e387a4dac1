#!/bin/bash
# gpurun (round 5): the drain on config 4 (scene in HBM with LDS caches: render_drain<HYB>) against the far pass's own
# launch, alternating in one process.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r05r"; mkdir -p "$OUT"
timeout -k 10 300 python scripts/ab.py --scene stress_100k --spp 100 --rounds 3 --variants "v3,v3@RTX_DRAIN=0" > "$OUT/c4.log" 2>&1 || { tail -5 "$OUT/c4.log"; exit 1; }
grep -h "sha256\|median" "$OUT/c4.log"
