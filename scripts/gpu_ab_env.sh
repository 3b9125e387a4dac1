#!/bin/bash
# gpurun: the full -m gpu suite, then bench lines of env variants on several workloads.
#   VARIANTS="RTX_COLLAPSE=0;RTX_COLLAPSE=1" WORKLOADS="|--scene stress_100k --spp 100" TAG=x
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-abenv}"; mkdir -p "$OUT"; export TMPDIR=/tmp
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
fi
IFS='|' read -ra WS <<< "${WORKLOADS:-}"
[ ${#WS[@]} -eq 0 ] && WS=("")
w=0
for args in "${WS[@]}"; do
  w=$((w+1))
  for rep in 1 2; do
    TAG="${TAG:-abenv}/w$w.r$rep" BENCH_ARGS="$args" LIMIT=${LIMIT:-300} bash scripts/gpu_variants.sh || exit 1
  done
done
