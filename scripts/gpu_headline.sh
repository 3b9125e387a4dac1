#!/bin/bash
# gpurun: the headline bench line, a rocprofv3 kernel trace of the same command, and the PMC
# passes (VALU issue, LDS, waits, HBM bytes, L2) of one timed launch, all under gpurun_out/$TAG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-head}
OUT="$PWD/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-}
timeout -k 10 400 python bench.py --steps ${STEPS:-5} --warmup 2 $ARGS > "$OUT/bench.json" 2> "$OUT/bench.err" && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --steps 3 --warmup 1 --no-cpu --no-hash $ARGS > "$OUT/bench_prof.log" 2>&1 && \
PMC_TAG=$TAG/pmc PMC_CMD="python bench.py --steps 1 --warmup 0 --no-cpu --no-hash $ARGS" bash scripts/gpu_pmc.sh
rc=$?
echo "exit=$rc"; tail -1 "$OUT/bench.json"
exit $rc
