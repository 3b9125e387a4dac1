#!/bin/bash
# gpurun (round 4): A/B of abl/librtx_$AB.so against the in-tree librtx.so on C2 (and C1, Cornell), alternating,
# then the parity tests named by $TESTS on the in-tree library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-r04j}"; mkdir -p "$OUT"; export TMPDIR=/tmp
line() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', d['ms_per_step'], d['kernel_ms_avg'], d.get('framebuffer_sha256_16'))"; }
for i in 1 2; do
  for lib in cur $AB; do
    [ $lib = cur ] && L="" || L="$PWD/abl/librtx_$lib.so"
    RTX_LIB=$L timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu > "$OUT/c2_${lib}_$i.json" 2> "$OUT/c2_${lib}_$i.err" || exit 1
    line "$OUT/c2_${lib}_$i.json" "c2 $lib $i"
    RTX_LIB=$L timeout -k 10 200 python bench.py --scene cornell_box --width 600 --spp 200 --steps 5 --warmup 1 --no-cpu > "$OUT/cb_${lib}_$i.json" 2> "$OUT/cb_${lib}_$i.err" || exit 1
    line "$OUT/cb_${lib}_$i.json" "cornell $lib $i"
  done
done
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$TESTS" > "$OUT/pytest_gpu.log" 2>&1
  rc=$?
  grep -E "passed|failed|error" "$OUT/pytest_gpu.log" | tail -6
  exit $rc
fi
