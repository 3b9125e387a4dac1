#!/bin/bash
# gpurun (round 5): the kernel trace of rank 0's rows of an 8-GPU run (where its time goes), and whole-frame
# parity of the round-5 library against the oracle (scripts/full_frame_parity.py): C1, C2, C4 every pixel,
# C3 every 4th row, C5 every 24th row.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/${FFP_TAG:-r05h}"; mkdir -p "$OUT"
for s in 0/8 0/4; do
  t=${s/\//of}
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$t" -o run --output-format csv -- python bench.py --no-cpu --shard $s \
      > "$OUT/shard_$t.json" 2> "$OUT/trace_$t.log" || { tail -5 "$OUT/trace_$t.log"; exit 1; }
  find "$OUT/trace_$t" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_$t.csv" \;
  echo "== shard $s"; head -5 "$OUT/kernel_stats_$t.csv" | cut -d, -f1-4
done
timeout -k 10 1000 python -u scripts/full_frame_parity.py C1 C2 C4 C3 C5 --stride C3=4 --stride C5=24 --out "$OUT/ffp.jsonl" \
    > "$OUT/ffp.log" 2>&1 || { tail -20 "$OUT/ffp.log"; exit 1; }
cat "$OUT/ffp.jsonl" | cut -c1-300
