#!/bin/bash
# gpurun: PC sampling (rocprofv3 beta, stochastic or host-trap) of one timed render, under
# gpurun_out/$TAG: where the render kernel's wave cycles sit, instruction by instruction.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source scripts/gpu_step.sh
TAG=${TAG:-pcs}; OUT="$PWD/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp
step 120 "$OUT/list.log" rocprofv3 -L
grep -i -A12 "pc sampling\|pc_sampling" "$OUT/list.log" | head -40
M=${METHOD:-stochastic}; U=${UNIT:-cycles}; I=${INTERVAL:-1048576}
step 300 "$OUT/run.log" rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $M --pc-sampling-unit $U \
    --pc-sampling-interval $I -d "$OUT/out" -o run --output-format csv -- python scripts/render_once.py --spp ${SPP:-20} ${ARGS:-}
tail -5 "$OUT/run.log"
ls -la "$OUT/out" 2>/dev/null | head
