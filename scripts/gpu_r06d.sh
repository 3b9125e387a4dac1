#!/bin/bash
# round 6: the paired walk — its parity tests and config 4's other tests, config 4 timed with records
# and with entries (RTX_W2=1 / 0, alternating), then the PMC A/B of the kernarg-reload and non-temporal builds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r06d"; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "paired or stress_100k or C4 or every_kernel" > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
for i in 1 2; do
  for w in 1 0; do
    RTX_W2=$w timeout -k 10 300 python bench.py --scene stress_100k --spp 100 --steps 3 --warmup 1 --no-cpu \
        > "$OUT/c4_w${w}_$i.json" 2> "$OUT/c4_w${w}_$i.err" || { tail "$OUT/c4_w${w}_$i.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['schedule']; print('w2=$w', d['ms_per_step'], d['kernel_ms_avg'], d['framebuffer_sha256_16'], d['node_visits_per_segment'], d['prim_tests_per_segment'], s.get('trav_lane_util'), s.get('lds_cache_hit_frac'))" "$OUT/c4_w${w}_$i.json"
  done
done
[ -n "$PMC" ] && { LIBS="$PMC" TAG=r06d bash scripts/gpu_pmc_libs.sh > "$OUT/pmc.txt" 2>&1 || exit 1; cut -c1-300 "$OUT/pmc.txt"; }


exit 0
