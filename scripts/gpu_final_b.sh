#!/bin/bash
# gpurun (the final library of a round, part 2): the configs table (gpu_configs.sh), every rank's shard
# (gpu_shards.sh) and the driver's round-end commands (gpu_driver.sh), on the profiles of part 1 (profiles/ in the
# tree sent).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${ROUND:-06}; OUT="$PWD/gpurun_out/final$R"; mkdir -p "$OUT"; export TMPDIR=/tmp
ROUND=$R bash scripts/gpu_configs.sh > "$OUT/configs.txt" 2>&1 || { tail -20 "$OUT/configs.txt"; exit 1; }
tail -2 "$OUT/configs.txt" | cut -c1-200
ROUND=$R bash scripts/gpu_shards.sh > "$OUT/shards.txt" 2>&1 || { tail -20 "$OUT/shards.txt"; exit 1; }
tail -2 "$OUT/shards.txt" | cut -c1-200
ROUND=$R bash scripts/gpu_driver.sh > "$OUT/driver.txt" 2>&1 || { tail -20 "$OUT/driver.txt"; exit 1; }
cat "$OUT/driver.txt" | cut -c1-300
