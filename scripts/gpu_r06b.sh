#!/bin/bash
# round 6: A/B of the kernarg-reload (fewer SGPR spills) and non-temporal colour-store builds against the in-tree
# library: kernel time (scripts/ab.py, alternating processes) and PMC counters per library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r06b"; mkdir -p "$OUT"; export TMPDIR=/tmp
LIBS="karg nt" AB_ARGS="--spp 100 --rounds 3 --variants v3" bash scripts/gpu_ab_libs.sh > "$OUT/ab.txt" 2>&1 && \
LIBS="karg nt" TAG=r06b bash scripts/gpu_pmc_libs.sh > "$OUT/pmc.txt" 2>&1
rc=$?
cat "$OUT/ab.txt" "$OUT/pmc.txt"
exit $rc
