#!/bin/bash
# gpurun (round 4): far-pass record claims by free lanes (in-tree) against 64-record units (abl/librtx_nofb.so),
# alternating, on C1, rank 0's rows at N = 4 / 8 and C2; then the tiered parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/r04o"; mkdir -p "$OUT"; export TMPDIR=/tmp
line() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', d['ms_per_step'], d['kernel_ms_avg'], d.get('framebuffer_sha256_16'))"; }
for i in 1 2; do
  for lib in cur nofb; do
    [ $lib = cur ] && L="" || L="$PWD/abl/librtx_$lib.so"
    RTX_LIB=$L timeout -k 10 120 python bench.py --width 400 --spp 100 --steps 20 --warmup 3 --no-cpu > "$OUT/c1_${lib}_$i.json" 2>/dev/null || exit 1
    line "$OUT/c1_${lib}_$i.json" "c1 $lib $i"
    for n in 4 8; do
      RTX_LIB=$L timeout -k 10 120 python bench.py --shard 0/$n --steps 5 --warmup 1 --no-cpu > "$OUT/s${n}_${lib}_$i.json" 2>/dev/null || exit 1
      line "$OUT/s${n}_${lib}_$i.json" "shard0of$n $lib $i"
    done
    RTX_LIB=$L timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu > "$OUT/c2_${lib}_$i.json" 2>/dev/null || exit 1
    line "$OUT/c2_${lib}_$i.json" "c2 $lib $i"
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "overflow or tier or config1 or config2_crop or shard or ties or nested or octant or deferred or smoke" > "$OUT/pytest_gpu.log" 2>&1
rc=$?
grep -E "passed|failed|error" "$OUT/pytest_gpu.log" | tail -4
exit $rc
