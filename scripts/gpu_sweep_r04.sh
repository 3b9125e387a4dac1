#!/bin/bash
# gpurun (round 4): knob A/B on the new margins, one call, best of 2 per setting (kernel ms from the
# bench line): the near region's growth for C2 and C4, the near pass's shading / primitive-batch thresholds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-sweep04}"; mkdir -p "$OUT"; export TMPDIR=/tmp
run() {  # name, env..., -- bench args
  local n=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  for rep in 1 2; do
    env "${envs[@]}" timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu --no-hash "$@" > "$OUT/$n.$rep.json" 2> "$OUT/$n.$rep.err" || return $?
    python -c "import json,sys; d=json.loads(open('$OUT/$n.$rep.json').read().strip().splitlines()[-1]); print('$n', '$rep', d['ms_per_step'], d['kernel_ms_avg'])"
  done
}
for g in 50 100 150 200 300; do run c2_grow$g RTX_NEAR_GROW=$g -- --spp 100 || exit $?; done
for g in 0 1 2 5; do run c4_grow$g RTX_NEAR_GROW=$g -- --scene stress_100k --spp 100 || exit $?; done
for t in 52 56 60; do for b in 8 12 16; do run c2_t${t}_b$b RTX_SHADE_THRESH=$t RTX_PRIM_BATCH=$b -- --spp 100 || exit $?; done; done
echo done
