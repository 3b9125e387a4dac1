#!/bin/bash
# gpurun: EVERY rank's rows of the 2/4/8-GPU headline runs rendered alone on this one GPU
# (bench.py --shard r/N: the timed kernel on rank r's rows y = r mod N, its tile shape), plus the one-process
# band assembly of 8 simulated bands (rtx_render with RTX_SIM_BANDS=8: device copies + de-interleave).
# Lines to gpurun_out/$TAG/shards.jsonl (scripts/scaling_prediction.py turns them into the predicted curve).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-shards${ROUND:-06}}; OUT="$PWD/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp
: > "$OUT/shards.jsonl"
for N in 2 4 8; do
  for ((r = 0; r < N; r++)); do
    timeout -k 10 200 python bench.py --shard $r/$N --no-cpu --steps 3 --warmup 1 > "$OUT/s${r}of$N.json" 2> "$OUT/s${r}of$N.err" || \
        { tail -5 "$OUT/s${r}of$N.err"; exit 1; }
    python - "$OUT/s${r}of$N.json" $r $N >> "$OUT/shards.jsonl" << 'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(json.dumps({"rank": int(sys.argv[2]), "world": int(sys.argv[3]), "ms_per_step": d["ms_per_step"],
                  "kernel_ms_avg": d.get("kernel_ms_avg"), "framebuffer_sha256_16": d.get("framebuffer_sha256_16"),
                  "librtx_sha256_16": d["roofline"].get("librtx_sha256_16") if d.get("roofline") else None,
                  "segments_per_sample": d.get("segments_per_sample"), "value": d["value"]}))
PY
    tail -1 "$OUT/shards.jsonl"
  done
done
RTX_SIM_BANDS=8 timeout -k 10 200 python bench.py --in-process --no-cpu --steps 3 --warmup 1 > "$OUT/sim8.json" 2> "$OUT/sim8.err" || \
    { tail -5 "$OUT/sim8.err"; exit 1; }
cut -c1-400 "$OUT/sim8.json"
