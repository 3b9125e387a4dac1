#!/bin/bash
# gpurun (round 5): the near pass's drain (render_drain, RTX_DRAIN) against the far pass's own launch, alternating in one
# process: C2, C1; rank 0 of 8 by bench.py --shard; then the tiered parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r05q"; mkdir -p "$OUT"
timeout -k 10 300 python scripts/ab.py --spp 500 --rounds 3 --variants "v3,v3@RTX_DRAIN=0" > "$OUT/c2.log" 2>&1 || { tail -5 "$OUT/c2.log"; exit 1; }
grep -h "sha256\|median" "$OUT/c2.log"
timeout -k 10 300 python scripts/ab.py --width 400 --spp 100 --rounds 5 --variants "v3,v3@RTX_DRAIN=0" > "$OUT/c1.log" 2>&1 || { tail -5 "$OUT/c1.log"; exit 1; }
grep -h "sha256\|median" "$OUT/c1.log"
for d in 1 0; do
  timeout -k 10 300 env RTX_DRAIN=$d python bench.py --shard 0/8 --steps 5 --warmup 1 --no-cpu > "$OUT/s08_$d.json" 2> "$OUT/s08_$d.err" || { tail -5 "$OUT/s08_$d.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/s08_$d.json')); print('shard0/8 drain=$d', d['ms_per_step'], d.get('kernel_ms_avg'), d['framebuffer_sha256_16'])"
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "tier or C1 or C2 or shard" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
