#!/bin/bash
# gpurun (round 4): C1 launch shape A/B — the near pass's grid (RTX_ITEM_GRID, % of the resident grid) and
# samples per unit (RTX_ITEM_SUB) — alternating, and C2 at 100 / 90 %.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r04l"; mkdir -p "$OUT"; export TMPDIR=/tmp
line() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); s=d['schedule']; print('$2', d['ms_per_step'], d['kernel_ms_avg'], s.get('idle_lane_frac'), d.get('framebuffer_sha256_16'))"; }
for i in 1 2; do
  for v in "100 0" "75 0" "50 0" "100 1" "100 4" "75 1"; do
    set -- $v
    RTX_ITEM_GRID=$1 RTX_ITEM_SUB=$2 timeout -k 10 120 python bench.py --width 400 --spp 100 --steps 20 --warmup 3 --no-cpu > "$OUT/c1_g$1_s$2_$i.json" 2> "$OUT/c1_g$1_s$2_$i.err" || exit 1
    line "$OUT/c1_g$1_s$2_$i.json" "c1 grid$1 sub$2 $i"
  done
  RTX_TIER=0 timeout -k 10 120 python bench.py --width 400 --spp 100 --steps 20 --warmup 3 --no-cpu > "$OUT/c1_notier_$i.json" 2> "$OUT/c1_notier_$i.err" || exit 1
  line "$OUT/c1_notier_$i.json" "c1 notier $i"
  for g in 100 90; do
    RTX_ITEM_GRID=$g timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu > "$OUT/c2_g${g}_$i.json" 2> "$OUT/c2_g${g}_$i.err" || exit 1
    line "$OUT/c2_g${g}_$i.json" "c2 grid$g $i"
  done
done
