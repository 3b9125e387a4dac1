#!/bin/bash
# round 6: the paired walk as records everywhere with its record-read estimate for the LDS cache (config 4, RTX_W2
# 1 / 0 alternating) and the kernarg-reload build against the in-tree library at the headline (scripts/ab.py, 500 spp)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r06e"; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "paired or stress_100k or C4" > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for i in 1 2; do
  for w in 1 0; do
    RTX_W2=$w timeout -k 10 300 python bench.py --scene stress_100k --spp 100 --steps 3 --warmup 1 --no-cpu \
        > "$OUT/c4_w${w}_$i.json" 2> "$OUT/c4_w${w}_$i.err" || { tail "$OUT/c4_w${w}_$i.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['schedule']; print('w2=$w', d['ms_per_step'], d['kernel_ms_avg'], d['framebuffer_sha256_16'], s.get('trav_lane_util'), s.get('lds_cache_hit_frac'))" "$OUT/c4_w${w}_$i.json"
  done
done
LIBS="karg" AB_ARGS="--spp 500 --rounds 2 --variants v3" bash scripts/gpu_ab_libs.sh > "$OUT/ab.txt" 2>&1 || exit 1
cat "$OUT/ab.txt"
