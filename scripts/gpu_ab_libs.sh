#!/bin/bash
# gpurun: A/B of library builds (abl/librtx_<name>.so, built here) against the in-tree
# librtx.so, one process each, alternating twice.  LIBS="s4 s2" AB_ARGS="--spp 100 ...".
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out"; mkdir -p "$OUT"; export TMPDIR=/tmp
ARGS=${AB_ARGS:---spp 100 --rounds 3 --variants v3}
for i in 1 2; do
  timeout -k 10 200 python scripts/ab.py $ARGS > "$OUT/ab_cur_$i.log" 2>&1 || exit 1
  echo "cur  $(grep "median\|sha256" "$OUT/ab_cur_$i.log" | head -4 | tr '\n' ' ')"
  for l in $LIBS; do
    RTX_LIB=$PWD/abl/librtx_$l.so timeout -k 10 200 python scripts/ab.py $ARGS > "$OUT/ab_${l}_$i.log" 2>&1 || exit 1
    echo "$l  $(grep "median\|sha256" "$OUT/ab_${l}_$i.log" | head -4 | tr '\n' ' ')"
  done
done
