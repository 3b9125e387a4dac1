#!/bin/bash
# gpurun (round 5): miss-phase threshold sweep (RTX_REFILL_HITS x shading threshold) on C2, the claim guard's cost
# (abl/librtx_noguard.so: -DRTX_CLAIM_GUARD=0), and C4 / C1 against round 4's library.  No tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-r05d}"; mkdir -p "$OUT"; export TMPDIR=/tmp
ab() {  # ab <log> [env...] -- args
  local log=$1; shift
  timeout -k 10 240 env "$@" > "$OUT/$log" 2>&1 || { tail -5 "$OUT/$log"; exit 1; }
  echo "== $log"; grep "median\|sha256" "$OUT/$log" | head -8
}
V="v3@RTX_REFILL_HITS=24,v3@RTX_REFILL_HITS=28,v3@RTX_REFILL_HITS=32,v3@RTX_REFILL_HITS=36,t52@RTX_REFILL_HITS=32,t60@RTX_REFILL_HITS=32"
for i in 1 2; do
  ab c2_cur_$i.log python scripts/ab.py --spp 500 --rounds 3 --variants $V
  ab c2_noguard_$i.log RTX_LIB=$PWD/abl/librtx_noguard.so python scripts/ab.py --spp 500 --rounds 3 --variants v3@RTX_REFILL_HITS=32,v3@RTX_CAM_POOL=0
  ab c2_r04_$i.log RTX_LIB=$PWD/abl/librtx_r04.so python scripts/ab.py --spp 500 --rounds 3 --variants v3
done
for i in 1 2; do
  ab c4_cur_$i.log python scripts/ab.py --scene stress_100k --spp 100 --rounds 2 --variants v3
  ab c4_noguard_$i.log RTX_LIB=$PWD/abl/librtx_noguard.so python scripts/ab.py --scene stress_100k --spp 100 --rounds 2 --variants v3
  ab c4_r04_$i.log RTX_LIB=$PWD/abl/librtx_r04.so python scripts/ab.py --scene stress_100k --spp 100 --rounds 2 --variants v3
done
ab c1_cur.log python scripts/ab.py --width 400 --spp 100 --rounds 5 --variants v3,v3@RTX_REFILL_HITS=32,v3@RTX_REFILL_HITS=24
ab c1_r04.log RTX_LIB=$PWD/abl/librtx_r04.so python scripts/ab.py --width 400 --spp 100 --rounds 5 --variants v3
