#!/bin/bash
# gpurun recipe: PMC A/B of library builds on one bench workload.  For the in-tree librtx.so ("cur") and each
# abl/librtx_<name>.so of LIBS: a VALU pass (SQ_INSTS_VALU/SALU, wave cycles and waits), a FETCH_SIZE and a WRITE_SIZE pass of
# one timed render (bench.py --steps 1 --warmup 0), summarised into gpurun_out/$TAG/valu.jsonl / traffic.jsonl
# (scripts/pmc_valu.py / pmc_traffic.py, keyed by each library's hash).
#   LIBS="karg nt" TAG=r06b WL="random_spheres:1920x1080x500" BARGS="" bash scripts/gpu_pmc_libs.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-pmclibs}; OUT="$PWD/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp
WL=${WL:-random_spheres:1920x1080x500}
PV="SQ_INSTS_VALU SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for l in cur ${LIBS:-}; do
  lib=$PWD/raytracer-go_amd/librtx.so; [ "$l" != cur ] && lib=$PWD/abl/librtx_$l.so; mkdir -p "$OUT/$l"
  cmd="python bench.py --steps 1 --warmup 0 --no-cpu --no-hash --no-verify ${BARGS:-}"
  for pass in valu fetch write; do
    case $pass in valu) P="$PV";; fetch) P="FETCH_SIZE";; write) P="WRITE_SIZE";; esac
    RTX_LIB=$lib timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $P -d "$OUT/$l/$pass" -o run --output-format csv \
        -- $cmd > "$OUT/$l/$pass.log" 2>&1 || { echo "$l $pass failed rc=$?"; exit 1; }
  done
  python scripts/pmc_valu.py "$OUT/$l/valu" "$OUT/valu.jsonl" --workload "$WL" --renders 1 --lib "$lib" \
      > "$OUT/$l/valu.json" || exit 1
  python scripts/pmc_traffic.py "$OUT/$l" "$OUT/traffic.jsonl" --workload "$WL" --renders 1 --lib "$lib" \
      > "$OUT/$l/traffic.json" || exit 1
  echo "$l: $(cut -c1-200 "$OUT/$l/valu.json")"
done
