#!/bin/bash
# gpurun: optionally a part of the GPU suite, then bench lines of environment variants on several workloads,
# alternating variants within each of two rounds (the same library; knobs read per render or per scene).
#   VARIANTS="RTX_TIER_QUADS=1|RTX_TIER_QUADS=0" WORKLOADS="--scene cornell_box --width 600 --spp 200|..." \
#   PYTEST_ARGS="tests/test_quads.py" TAG=x bash scripts/gpu_ab_env.sh       (VARIANTS: '|'-separated, ';' within)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-abenv}"; mkdir -p "$OUT"; export TMPDIR=/tmp
if [ -n "$PYTEST_ARGS" ]; then
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest $PYTEST_ARGS -x -v --timeout 300 --timeout-method thread \
      > "$OUT/pytest.log" 2>&1
  rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "^E |FAILED" "$OUT/pytest.log" | head -20; exit $rc; }
fi
IFS='|' read -ra VS <<< "${VARIANTS:-}"
IFS='|' read -ra WS <<< "${WORKLOADS:-}"
[ ${#WS[@]} -eq 0 ] && WS=("")
w=0
for args in "${WS[@]}"; do
  w=$((w+1))
  for rep in 1 2; do
    v=0
    for var in "${VS[@]}"; do
      v=$((v+1))
      f="$OUT/w$w.v$v.r$rep"
      env $(echo "$var" | tr ';' ' ') timeout -k 10 ${LIMIT:-300} python bench.py --no-cpu --steps ${STEPS:-5} \
          --warmup 1 $args > "$f.json" 2> "$f.err" || { tail -5 "$f.err"; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); s=d.get('schedule',{}); print(sys.argv[2], '|', sys.argv[3], '|', d['ms_per_step'], d['kernel_ms_avg'], d['framebuffer_sha256_16'], d['node_visits_per_segment'], d['prim_tests_per_segment'], d['walk_layout'][:60])" "$f.json" "$args" "$var"
    done
  done
done
