#!/bin/bash
# round 6: the whole GPU suite and smoke on the karg-reload default build, then config 4 with the drain for scenes
# in HBM (abl/librtx_hybdrain.so) against the in-tree library, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r06f"; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
for i in 1 2; do
  for l in cur hybdrain; do
    lib=$PWD/raytracer-go_amd/librtx.so; [ $l != cur ] && lib=$PWD/abl/librtx_$l.so
    RTX_LIB=$lib timeout -k 10 300 python bench.py --scene stress_100k --spp 100 --steps 3 --warmup 1 --no-cpu \
        > "$OUT/c4_${l}_$i.json" 2> "$OUT/c4_${l}_$i.err" || { tail "$OUT/c4_${l}_$i.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('$l', d['ms_per_step'], d['kernel_ms_avg'], d['framebuffer_sha256_16'])" "$OUT/c4_${l}_$i.json"
  done
done
