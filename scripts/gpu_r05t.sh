#!/bin/bash
# gpurun (round 5, drain library): the kernel trace of the driver's default bench command, the default bench line on
# the fresh profiles, every rank's shard (scripts/gpu_shards_r05.sh), the whole GPU suite and smoke.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r05t"; mkdir -p "$OUT"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python bench.py --no-cpu \
    > "$OUT/bench_under_rocprof.json" 2> "$OUT/trace.log" || { tail -5 "$OUT/trace.log"; exit 1; }
find "$OUT/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
head -8 "$OUT/kernel_stats.csv" | cut -c1-200
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('bench', d['value'], d['ms_per_step'], d['framebuffer_sha256_16'], d['roofline']['frac'], d['roofline'].get('lane_frac'), d['cpu_baseline']['value'])"
TAG=shards05 bash scripts/gpu_shards_r05.sh || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 && \
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?
grep -E "passed|failed|error" "$OUT/pytest_gpu.log" | tail -3; tail -1 "$OUT/smoke.log"
exit $rc
