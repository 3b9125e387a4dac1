#!/bin/bash
# gpurun (round 5): miss phases x shading threshold, finer (C2), and the claim guard's flag as an SGPR of its
# own (in tree) / bit 31 of the loop counter (abl/librtx_kiter.so) / no guard (abl/librtx_noguard.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-r05e}"; mkdir -p "$OUT"; export TMPDIR=/tmp
ab() {  # ab <log> [env...] -- args
  local log=$1; shift
  timeout -k 10 240 env "$@" > "$OUT/$log" 2>&1 || { tail -5 "$OUT/$log"; exit 1; }
  echo "== $log"; grep "median\|sha256" "$OUT/$log" | head -9
}
V="v3@RTX_REFILL_HITS=36,v3@RTX_REFILL_HITS=40,t52@RTX_REFILL_HITS=36,t52@RTX_REFILL_HITS=40,t48@RTX_REFILL_HITS=32,t48@RTX_REFILL_HITS=36,t48@RTX_REFILL_HITS=40,t44@RTX_REFILL_HITS=36"
W="v3@RTX_REFILL_HITS=36,t52@RTX_REFILL_HITS=36"
for i in 1 2; do
  ab c2_cur_$i.log python scripts/ab.py --spp 500 --rounds 3 --variants $V
  ab c2_kiter_$i.log RTX_LIB=$PWD/abl/librtx_kiter.so python scripts/ab.py --spp 500 --rounds 3 --variants $W
  ab c2_noguard_$i.log RTX_LIB=$PWD/abl/librtx_noguard.so python scripts/ab.py --spp 500 --rounds 3 --variants $W
done
