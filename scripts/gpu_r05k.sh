#!/bin/bash
# gpurun (round 5): the striped library (per-tile row base: affine; per-lane mapping: stripegen) against the one
# before stripes (prestripe) on C2 in one call; the
# advisor's mid-size LDS cache A/B on an UNTIERED config-4 render (RTX_TIER=0: the caller's tree alone, where the
# 8-wave / 12-wave switch applies): RTX_HOT_ENTRIES=1280 in tree (12-wave) against HOT_B = 32 KB (8-wave); then the
# driver's default bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r05k"; mkdir -p "$OUT"
for i in 1 2; do
  for lib in affine stripegen prestripe; do
    L="RTX_LIB=$PWD/abl/librtx_$lib.so"
    timeout -k 10 240 env $L python scripts/ab.py --spp 500 --rounds 3 --variants v3 > "$OUT/c2_${lib}_$i.log" 2>&1 || { tail -5 "$OUT/c2_${lib}_$i.log"; exit 1; }
    echo "$lib $(grep median "$OUT/c2_${lib}_$i.log" | head -1)"
  done
done
for i in 1 2; do
  for lib in cur hotb32k; do
    L=""; [ $lib != cur ] && L="RTX_LIB=$PWD/abl/librtx_$lib.so"
    timeout -k 10 240 env $L RTX_TIER=0 RTX_HOT_ENTRIES=1280 RTX_DEBUG_LAUNCH=1 python scripts/ab.py --scene stress_100k --spp 100 --rounds 2 \
        --variants v3 > "$OUT/c4u_${lib}_$i.log" 2>&1 || { tail -5 "$OUT/c4u_${lib}_$i.log"; exit 1; }
    echo "$lib $(grep 'rtx v3' "$OUT/c4u_${lib}_$i.log" | tail -1 | cut -c1-70) $(grep median "$OUT/c4u_${lib}_$i.log" | head -1)"
  done
done
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('bench', d['value'], d['ms_per_step'], d['framebuffer_sha256_16'], d['roofline']['frac'], d['roofline'].get('lane_frac'), d['cpu_baseline']['value'])"
