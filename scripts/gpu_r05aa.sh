#!/bin/bash
# gpurun (round 5): config 4 with the pipelined HBM walk (traverse_loop_pipe, RTX_HYB_PIPE) against the walk that waits
# per step, the same scene (1024-entry cache) alternating in one process; then the old default (2560-entry cache, no pipe).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r05aa"; mkdir -p "$OUT"
timeout -k 10 300 python scripts/ab.py --scene stress_100k --spp 100 --rounds 3 --variants "v3,v3@RTX_HYB_PIPE=0" > "$OUT/c4.log" 2>&1 || { tail -5 "$OUT/c4.log"; exit 1; }
grep -h "sha256\|median" "$OUT/c4.log"
RTX_HOT_ENTRIES=2560 RTX_HYB_PIPE=0 timeout -k 10 300 python scripts/ab.py --scene stress_100k --spp 100 --rounds 3 --variants "v3" > "$OUT/c4_old.log" 2>&1 || { tail -5 "$OUT/c4_old.log"; exit 1; }
grep -h "sha256\|median" "$OUT/c4_old.log"
