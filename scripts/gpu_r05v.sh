#!/bin/bash
# gpurun (round 5): C2 WRITE_SIZE with the drain at region sizes 20000 (RTX_DEFER_CAP = 512 x 20000) and the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r05v"; mkdir -p "$OUT"
for cap in 10240000 40960000; do
  RTX_DEFER_CAP=$cap timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/c$cap" -o run --output-format csv -- \
      python bench.py --steps 1 --warmup 0 --no-cpu --no-hash > "$OUT/c$cap.log" 2>&1 || { tail -5 "$OUT/c$cap.log"; exit 1; }
  python - "$OUT/c$cap" $cap << 'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
tot = collections.defaultdict(float)
for r in csv.DictReader(open(f)):
    tot[r["Kernel_Name"][:40]] += float(r["Counter_Value"]) * 1024 / 1e9
print(sys.argv[2], {k: round(v, 3) for k, v in tot.items() if v > 0.1})
PY
done
