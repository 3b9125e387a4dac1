#!/bin/bash
# gpurun (round 5): bench.py with the one-rank steps enqueued back to back (C2 default, C1, rank 0 of 8).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r05ac"; mkdir -p "$OUT"
timeout -k 10 300 python bench.py > "$OUT/c2.json" 2> "$OUT/c2.err" || { tail -20 "$OUT/c2.err"; exit 1; }
timeout -k 10 300 python bench.py --width 400 --spp 100 --steps 20 --warmup 2 > "$OUT/c1.json" 2> "$OUT/c1.err" || { tail -20 "$OUT/c1.err"; exit 1; }
timeout -k 10 300 python bench.py --shard 0/8 --no-cpu > "$OUT/s08.json" 2> "$OUT/s08.err" || { tail -20 "$OUT/s08.err"; exit 1; }
for f in c2 c1 s08; do python -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', d['value'], d['ms_per_step'], d['kernel_ms_avg'], d['framebuffer_sha256_16'], d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'))"; done
