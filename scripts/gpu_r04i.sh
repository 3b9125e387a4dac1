#!/bin/bash
# gpurun (round 4): the 80 KB LDS cache (2560 entries) against 2048 entries on config 4 (same build,
# RTX_HOT_ENTRIES), alternating, then the whole GPU suite and smoke on this library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r04i"; mkdir -p "$OUT"; export TMPDIR=/tmp
line() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', d['ms_per_step'], d['kernel_ms_avg'], d['schedule'].get('lds_cache_hit_frac'), d.get('framebuffer_sha256_16'))"; }
for i in 1 2; do
  for hot in 2048 2560; do
    RTX_HOT_ENTRIES=$hot timeout -k 10 200 python bench.py --scene stress_100k --spp 100 --steps 5 --warmup 1 --no-cpu > "$OUT/c4_h${hot}_$i.json" 2> "$OUT/c4_h${hot}_$i.err" || exit 1
    line "$OUT/c4_h${hot}_$i.json" "c4 hot$hot $i"
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 && \
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?
grep -E "passed|failed|error" "$OUT/pytest_gpu.log" | tail -6; tail -2 "$OUT/smoke.log"
exit $rc
