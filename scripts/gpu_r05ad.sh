#!/bin/bash
# gpurun (round 5): one launch for a chunk's counters (chunk_start), the redo bits cleared by reduce_samples: the tiered
# GPU tests (parity, queue overflow and the redo bits' path, drain, id limit, claim guard), then the bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r05ad"; mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_claim_guard.py tests/test_render_entry.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python bench.py > "$OUT/c2.json" 2> "$OUT/c2.err" || { tail -20 "$OUT/c2.err"; exit 1; }
timeout -k 10 300 python bench.py --width 400 --spp 100 --steps 20 --warmup 2 > "$OUT/c1.json" 2> "$OUT/c1.err" || { tail -20 "$OUT/c1.err"; exit 1; }
for f in c2 c1; do python -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', d['value'], d['ms_per_step'], d['kernel_ms_avg'], d['framebuffer_sha256_16'], (d.get('cpu_baseline') or {}).get('value'))"; done
