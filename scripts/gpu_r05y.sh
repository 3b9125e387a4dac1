#!/bin/bash
# gpurun (round 5): samples per unit (RTX_ITEM_SUB) with the drain: C1, rank 0 of 8, C2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r05y"; mkdir -p "$OUT"
timeout -k 10 300 python scripts/ab.py --width 400 --spp 100 --rounds 5 \
    --variants "v3,v3@RTX_ITEM_SUB=4,v3@RTX_ITEM_SUB=8,v3@RTX_ITEM_SUB=16,v3@RTX_ITEM_SUB=2" > "$OUT/c1.log" 2>&1 || { tail -5 "$OUT/c1.log"; exit 1; }
grep -h "sha256\|median" "$OUT/c1.log"
for s in 0 4 16 8; do
  E=""; [ $s != 0 ] && E="RTX_ITEM_SUB=$s"
  timeout -k 10 300 env $E python bench.py --shard 0/8 --steps 5 --warmup 1 --no-cpu > "$OUT/s08_$s.json" 2> "$OUT/s08_$s.err" || { tail -5 "$OUT/s08_$s.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/s08_$s.json')); print('shard0/8 sub=$s', d['ms_per_step'], d.get('kernel_ms_avg'), d['framebuffer_sha256_16'])"
done
timeout -k 10 300 python scripts/ab.py --spp 500 --rounds 2 --variants "v3,v3@RTX_ITEM_SUB=32,v3@RTX_ITEM_SUB=8" > "$OUT/c2.log" 2>&1 || { tail -5 "$OUT/c2.log"; exit 1; }
grep -h "sha256\|median" "$OUT/c2.log"
