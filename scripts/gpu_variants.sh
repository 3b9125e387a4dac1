#!/bin/bash
# gpurun: bench lines of several variants (env assignments per line in $VARIANTS, ';'-separated),
# each under its own time limit; output gpurun_out/$TAG/v<i>.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-variants}"; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
IFS=';' read -ra VS <<< "$VARIANTS"
for v in "${VS[@]}"; do
  i=$((i+1))
  echo "variant $i: $v" > "$OUT/v$i.cmd"
  timeout -k 10 ${LIMIT:-240} env $v python bench.py --no-cpu ${BENCH_ARGS:-} > "$OUT/v$i.json" 2> "$OUT/v$i.err" || { echo "variant $i failed"; exit 1; }
  python - "$OUT/v$i.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:50s} {d['ms_per_step']:9.3f} ms  {d['value']:10.1f} {d['unit']}  nv/seg {d['node_visits_per_segment']}  hash {d.get('framebuffer_sha256_16')}  {d.get('walk_layout')}")
PY
done
