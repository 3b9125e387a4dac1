#!/bin/bash
# gpurun (round 4): env-knob sweep for rank 0's rows at N = 8 (unit size, shade threshold, primitive batch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r04p"; mkdir -p "$OUT"; export TMPDIR=/tmp
line() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', d['ms_per_step'], d['kernel_ms_avg'], d['schedule'].get('idle_lane_frac'), d.get('framebuffer_sha256_16'))"; }
for i in 1 2; do
  for v in "X=0" "RTX_ITEM_SUB=16" "RTX_ITEM_SUB=4" "RTX_SHADE_THRESH=52" "RTX_SHADE_THRESH=60" "RTX_PRIM_BATCH=16" "RTX_PRIM_BATCH=8"; do
    env $v timeout -k 10 120 python bench.py --shard 0/8 --steps 5 --warmup 1 --no-cpu > "$OUT/s8_${v}_$i.json" 2>/dev/null || exit 1
    line "$OUT/s8_${v}_$i.json" "s8 $v $i"
  done
done
