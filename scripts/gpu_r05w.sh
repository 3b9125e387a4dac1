#!/bin/bash
# gpurun (round 5): C2 WRITE_SIZE per kernel, drain on/off, with the queue (default) and without (RTX_DEFER_CAP=0: every
# deferred path to the redo pass) — where the drain's extra HBM writes come from.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r05w"; mkdir -p "$OUT"
for d in 1 0; do
  for cap in 0 default; do
    E="RTX_DRAIN=$d"; [ $cap != default ] && E="$E RTX_DEFER_CAP=$cap"
    timeout -s KILL 200 env $E rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/d${d}c$cap" -o run --output-format csv -- \
        python bench.py --steps 1 --warmup 0 --no-cpu --no-hash > "$OUT/d${d}c$cap.log" 2>&1 || { tail -5 "$OUT/d${d}c$cap.log"; exit 1; }
    python - "$OUT/d${d}c$cap" "drain=$d cap=$cap" << 'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
tot = collections.defaultdict(float)
for r in csv.DictReader(open(f)):
    tot[r["Kernel_Name"][:60]] += float(r["Counter_Value"]) * 1024 / 1e9
print(sys.argv[2], {k: round(v, 3) for k, v in tot.items() if v > 0.05})
PY
  done
done
