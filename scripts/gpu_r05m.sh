#!/bin/bash
# gpurun (round 5): stripe height of the shards, EVERY rank (the slowest one is the N-GPU step): N = 8 and N = 4,
# stripes of 1 (single rows, round 4's layout), 2, 4 and 8 rows; bench.py --shard r/N --stripe S alone on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r05m"; mkdir -p "$OUT"; export TMPDIR=/tmp
: > "$OUT/stripes.jsonl"
for N in 8 4; do
  for S in 1 2 4 8; do
    for ((r = 0; r < N; r++)); do
      t=s${r}of${N}_S$S
      timeout -k 10 200 python bench.py --shard $r/$N --stripe $S --no-cpu --steps 3 --warmup 1 > "$OUT/$t.json" 2> "$OUT/$t.err" || { tail -5 "$OUT/$t.err"; exit 1; }
      python -c "import json; d=json.load(open('$OUT/$t.json')); print(json.dumps({'rank': $r, 'world': $N, 'stripe': $S, 'kernel_ms_avg': d.get('kernel_ms_avg'), 'ms_per_step': d['ms_per_step'], 'framebuffer_sha256_16': d['framebuffer_sha256_16']}))" >> "$OUT/stripes.jsonl"
    done
    python -c "
import json
rows=[json.loads(l) for l in open('$OUT/stripes.jsonl')]
ms=[r['kernel_ms_avg'] for r in rows if r['world']==$N and r['stripe']==$S]
print('N=$N S=$S max %.3f mean %.3f min %.3f' % (max(ms), sum(ms)/len(ms), min(ms)))"
  done
done
