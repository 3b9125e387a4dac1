#!/bin/bash
# gpurun (round 5): WRITE_SIZE / FETCH_SIZE of C2 with the drain and with the far pass's own launch (RTX_DRAIN=0), same library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r05u"; mkdir -p "$OUT"
for d in 1 0; do
  for P in WRITE_SIZE FETCH_SIZE; do
    RTX_DRAIN=$d timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $P -d "$OUT/d$d/$P" -o run --output-format csv -- \
        python bench.py --steps 1 --warmup 0 --no-cpu --no-hash > "$OUT/d${d}_$P.log" 2>&1 || { tail -5 "$OUT/d${d}_$P.log"; exit 1; }
  done
  python scripts/pmc_traffic.py "$OUT/d$d" "$OUT/traffic_d$d.json" --workload "random_spheres:1920x1080x500/drain$d" --renders 1 | cut -c1-600
done
