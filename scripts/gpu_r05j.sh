#!/bin/bash
# gpurun (round 5, final library): the LDS-cache size A/B the advisor asked for (config 4 with a mid-size 1280-entry
# cache: the in-tree 12-wave kernel against a HOT_B = 32 KB build whose three 8-wave workgroups per CU take it),
# then the measurement set: kernel trace of the default bench command, PMC profiles of every workload, all 14
# shards (8-row stripes), 8 simulated bands in one process.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r05j"; mkdir -p "$OUT"
for i in 1 2; do
  for lib in cur hotb32k; do
    L=""; [ $lib = hotb32k ] && L="RTX_LIB=$PWD/abl/librtx_hotb32k.so"
    timeout -k 10 240 env $L RTX_HOT_ENTRIES=1280 RTX_DEBUG_LAUNCH=1 python scripts/ab.py --scene stress_100k --spp 100 --rounds 2 --variants v3 \
        > "$OUT/c4_hot1280_${lib}_$i.log" 2>&1 || { tail -5 "$OUT/c4_hot1280_${lib}_$i.log"; exit 1; }
    echo "$lib $(grep -m1 'waves/wg' "$OUT/c4_hot1280_${lib}_$i.log" | cut -c1-60) $(grep median "$OUT/c4_hot1280_${lib}_$i.log" | head -1)"
  done
done
bash scripts/gpu_r05g.sh
