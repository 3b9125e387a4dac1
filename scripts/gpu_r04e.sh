#!/bin/bash
# gpurun (round 4): the near walk's FMA slab form A/B (in-tree librtx.so vs abl/librtx_nofma.so, built with
# -DRTX_NEAR_FMA=0), C2 and C4, alternating, two rounds; then the tier / parity tests on the new build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r04e"; mkdir -p "$OUT"; export TMPDIR=/tmp
line() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', d['ms_per_step'], d['kernel_ms_avg'], d['node_visits_per_segment'], d['prim_tests_per_segment'], d.get('framebuffer_sha256_16'))"; }
for i in 1 2; do
  for v in fma nofma; do
    L=""; [ $v = nofma ] && L="$PWD/abl/librtx_nofma.so"
    RTX_LIB=$L timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu > "$OUT/c2_${v}_$i.json" 2> "$OUT/c2_${v}_$i.err" || exit 1
    line "$OUT/c2_${v}_$i.json" "c2 $v $i"
    RTX_LIB=$L timeout -k 10 200 python bench.py --scene stress_100k --spp 100 --steps 3 --warmup 1 --no-cpu > "$OUT/c4_${v}_$i.json" 2> "$OUT/c4_${v}_$i.err" || exit 1
    line "$OUT/c4_${v}_$i.json" "c4 $v $i"
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    -k "rows_vs_oracle or tier or ties or stress_100k or overflow or octant or config or go_sequence or nested" > "$OUT/pytest_gpu.log" 2>&1
rc=$?
grep -E "passed|failed|error" "$OUT/pytest_gpu.log" | tail -6
exit $rc
