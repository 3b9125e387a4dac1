#!/bin/bash
# gpurun (round 5): 8-row stripes for the shards — the whole GPU suite, then rank 0's (and rank N-1's) rows of
# 2/4/8-GPU runs rendered alone with single-row interleave (--stripe 1, round 4's layout) and 8-row stripes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-r05i}"; mkdir -p "$OUT"; export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
grep -E "passed|failed|error" "$OUT/pytest_gpu.log" | tail -4
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" "$OUT/pytest_gpu.log" | head -100; exit $rc; }
fi
for i in 1 2; do
for s in 0/8 7/8 0/4 0/2; do
  for st in 1 8; do
    t=${s/\//of}_s$st
    timeout -k 10 200 python bench.py --shard $s --stripe $st --no-cpu --steps 3 --warmup 1 > "$OUT/$t.json" 2> "$OUT/$t.err" || { tail -5 "$OUT/$t.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/$t.json')); print('$t', d['ms_per_step'], d.get('kernel_ms_avg'), d['framebuffer_sha256_16'])"
  done
done
done
