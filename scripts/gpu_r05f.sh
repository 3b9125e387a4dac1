#!/bin/bash
# gpurun (round 5): the whole GPU suite on the pooled library (counting kernels pooled too), smoke, the
# default bench line, and C2 / C4 / C1 / Cornell against round 4's library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-r05f}"; mkdir -p "$OUT"; export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 && \
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?
grep -E "passed|failed|error" "$OUT/pytest_gpu.log" | tail -4; tail -1 "$OUT/smoke.log"
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" "$OUT/pytest_gpu.log" | head -100; exit $rc; }
fi
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('bench', d['value'], d['ms_per_step'], d['framebuffer_sha256_16'], d.get('schedule'))"
ab() {
  local log=$1; shift
  timeout -k 10 240 env "$@" > "$OUT/$log" 2>&1 || { tail -5 "$OUT/$log"; exit 1; }
  echo "== $log"; grep "median\|sha256\|trav-lane" "$OUT/$log" | head -6
}
ab knobs.log python scripts/ab.py --spp 500 --rounds 3 --variants "v3,v3@RTX_ITEM_SUB=8,v3@RTX_ITEM_SUB=32,v3@RTX_PRIM_BATCH=8,v3@RTX_PRIM_BATCH=16,v3@RTX_REFILL_HITS=34,v3@RTX_REFILL_HITS=38"
for sc in "--spp 500" "--scene stress_100k --spp 100" "--width 400 --spp 100 --rounds 5" "--scene cornell_box --width 600 --spp 200"; do
  ab cur.log python scripts/ab.py $sc --variants v3
  ab r04.log RTX_LIB=$PWD/abl/librtx_r04.so python scripts/ab.py $sc --variants v3
done
