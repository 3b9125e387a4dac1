#!/bin/bash
# gpurun: the tiered walk — smoke, a subset of the parity tests, and the C2 bench
# with and without tiers (RTX_TIER=0), under gpurun_out/$TAG.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source scripts/gpu_step.sh
TAG=${TAG:-tier}; OUT="$PWD/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp
step 240 "$OUT/smoke.log" python -c "import __graft_entry__ as g; g.smoke()"
tail -2 "$OUT/smoke.log"
step 400 "$OUT/pytest.log" python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_random_scenes.py} -m gpu -x -q \
    --timeout 150 --timeout-method thread -k "${KSEL:-not full_frame and not rows_vs}"
tail -3 "$OUT/pytest.log"
for t in 0 1; do
    RTX_TIER=$t step 200 "$OUT/bench_t$t.json" python bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu ${BENCH_ARGS:-}
    python -c "import json,sys; d=json.loads(open('$OUT/bench_t$t.json').read().strip().splitlines()[-1]); print('tier', $t, d['ms_per_step'], d['framebuffer_sha256_16'], d['walk_layout'], d.get('node_visits_per_segment'), d.get('prim_tests_per_segment'))" || tail -5 "$OUT/bench_t$t.json"
done
if [ -n "$DIFF" ]; then
    step 300 "$OUT/diff_c2.log" python scripts/tier_diff.py random_spheres 1920 500 "$OUT/diff_c2.json"
    tail -1 "$OUT/diff_c2.log" | cut -c1-600
fi
if [ -n "$SPLIT" ]; then
    for nt in "" "--no-tier"; do
        step 200 "$OUT/split$nt.json" python scripts/timing_split.py --spp 100 $nt
        tail -1 "$OUT/split$nt.json"
    done
fi
if [ -n "$PROF" ]; then
    step 300 "$OUT/prof.log" rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
        python scripts/render_once.py --spp 500
    python -c "
import csv
for r in csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')): print(r['Name'][:70], r['Calls'], r['AverageNs'])" || true
fi
