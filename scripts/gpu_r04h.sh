#!/bin/bash
# gpurun (round 4): tile-shape A/B for one rank's rows at N = 4 and 8 (16 x 4 tiles, the new default there,
# against 8 x 8), then the shard / tile parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r04h"; mkdir -p "$OUT"; export TMPDIR=/tmp
line() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', d['ms_per_step'], d['kernel_ms_avg'], d['schedule'].get('trav_lane_util'), d.get('framebuffer_sha256_16'))"; }
for i in 1 2; do
  for n in 4 8; do
    for tw in 8 16 32; do
      RTX_TILE_W=$tw timeout -k 10 200 python bench.py --shard 0/$n --steps 5 --warmup 1 --no-cpu > "$OUT/s${n}_t${tw}_$i.json" 2> "$OUT/s${n}_t${tw}_$i.err" || exit 1
      line "$OUT/s${n}_t${tw}_$i.json" "shard0of$n tile$tw $i"
    done
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "shard or tile or band or v3" > "$OUT/pytest_gpu.log" 2>&1
rc=$?
grep -E "passed|failed|error" "$OUT/pytest_gpu.log" | tail -6
exit $rc
