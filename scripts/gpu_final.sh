#!/bin/bash
# gpurun: the round's final evidence in one call, under gpurun_out/$TAG:
#   PMC passes of one timed C2 step -> valu / traffic summaries (also copied into profiles/ on the box,
#   so the bench line below derives roofline.frac from them), the bench line, a rocprofv3 kernel
#   trace of the same command, the near-region A/B, the GPU test suite + smoke, the config lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source scripts/gpu_step.sh
TAG=${TAG:-final}; OUT="$PWD/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp
W="random_spheres:1920x1080x500"
PMC_TAG=$TAG/pmc PMC_CMD="python bench.py --steps 1 --warmup 0 --no-cpu --no-hash" step 900 "$OUT/pmc.log" bash scripts/gpu_pmc.sh
python scripts/pmc_valu.py "$OUT/pmc" "$OUT/valu_r03.json" --workload $W > "$OUT/valu.log" 2>&1 && \
python scripts/pmc_traffic.py "$OUT/pmc" "$OUT/traffic_r03.json" --workload $W > "$OUT/traffic.log" 2>&1 && \
cp "$OUT/valu_r03.json" "$OUT/traffic_r03.json" profiles/
cat "$OUT/valu.log" "$OUT/traffic.log" | cut -c1-300
step 400 "$OUT/bench.json" python bench.py --steps ${STEPS:-5} --warmup 2
tail -1 "$OUT/bench.json" | cut -c1-400
step 400 "$OUT/bench_prof.log" rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --steps 3 --warmup 1 --no-cpu --no-hash
RTX_NEAR_GROW=25 step 300 "$OUT/bench_grow25.json" python bench.py --steps 3 --warmup 1 --no-cpu
RTX_TIER=0 step 300 "$OUT/bench_notier.json" python bench.py --steps 3 --warmup 1 --no-cpu
for f in bench_grow25 bench_notier; do tail -1 "$OUT/$f.json" | cut -c1-200; done
[ -n "$SKIP_TESTS" ] || step 1100 "$OUT/pytest_gpu.log" python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
grep -E "passed|failed" "$OUT/pytest_gpu.log" | tail -2
[ -n "$SKIP_TESTS" ] || step 200 "$OUT/smoke.log" python -c "import __graft_entry__ as g; g.smoke()"
tail -1 "$OUT/smoke.log"
[ -n "$SKIP_CONFIGS" ] || TAG=$TAG/configs step 1500 "$OUT/configs.log" bash scripts/gpu_configs.sh
tail -2 "$OUT/configs.log"
