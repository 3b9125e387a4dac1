#!/bin/bash
# round 6: PMC counters of the kernarg-reload and non-temporal colour-store builds against the in-tree library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r06c"; mkdir -p "$OUT"; export TMPDIR=/tmp
LIBS="karg nt" TAG=r06c bash scripts/gpu_pmc_libs.sh > "$OUT/pmc.txt" 2>&1
rc=$?
cat "$OUT/pmc.txt"
exit $rc
