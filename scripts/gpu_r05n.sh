#!/bin/bash
# gpurun (round 5, final library; single-row shards by default again): the C2 kernel time, the measurement set
# (kernel trace of the default bench, PMC profiles of every workload, all 14 striped shards, 8 simulated bands), the
# default bench line on the fresh profiles, and the whole GPU suite + smoke.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/r05n"; mkdir -p "$OUT"
for i in 1 2; do
  for lib in cur; do
    L=""; [ $lib != cur ] && L="RTX_LIB=$PWD/abl/librtx_$lib.so"
    timeout -k 10 240 env $L python scripts/ab.py --spp 500 --rounds 3 --variants v3 > "$OUT/c2_${lib}_$i.log" 2>&1 || { tail -5 "$OUT/c2_${lib}_$i.log"; exit 1; }
    echo "$lib $(grep median "$OUT/c2_${lib}_$i.log" | head -1)"
  done
done
TRACE_TAG=r05n_trace bash scripts/gpu_r05g.sh || exit 1
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('bench', d['value'], d['ms_per_step'], d['framebuffer_sha256_16'], d['roofline']['frac'], d['roofline'].get('lane_frac'), d['cpu_baseline']['value'])"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 && \
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?
grep -E "passed|failed|error" "$OUT/pytest_gpu.log" | tail -3; tail -1 "$OUT/smoke.log"
exit $rc
