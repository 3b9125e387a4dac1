#!/bin/bash
# gpurun: PMC profiles of every bench workload on this library — the configs of SURVEY §8(d),
# the Cornell box, and rank 0's rows of the 2/4/8-GPU headline runs (bench.py --shard 0/N) — then the
# bench line of each, whose roofline.frac derives from them.  Per workload three rocprofv3 passes of one
# timed render (bench.py --steps 1 --warmup 0): VALU + wave-state counters, FETCH_SIZE, WRITE_SIZE.
# Summaries append to gpurun_out/$TAG/{valu,traffic}_r05.jsonl, copied into profiles/ on the box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${ROUND:-06}; TAG=${TAG:-prof$R}; OUT="$PWD/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp
PV="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
declare -a NAMES ARGS KEYS
add() { NAMES+=("$1"); KEYS+=("$2"); ARGS+=("$3"); }
add c2 "random_spheres:1920x1080x500" ""
add c1 "random_spheres:400x225x100" "--width 400 --spp 100"
add c3 "random_spheres:1920x1080x2000" "--spp 2000"
add c4 "stress_100k:1920x1080x100" "--scene stress_100k --spp 100"
add c5 "earth_dielectric:3840x2160x1000" "--scene earth_dielectric --width 3840 --spp 1000"
add cornell "cornell_box:600x600x200" "--scene cornell_box --width 600 --spp 200"
add quad "quad_demo:400x225x100" "--scene quad_demo --width 400 --spp 100"
add perlin "perlin_demo:400x225x100" "--scene perlin_demo --width 400 --spp 100"
add light "simple_light_demo:400x225x500" "--scene simple_light_demo --width 400 --spp 500"
add c2_r0of2 "random_spheres:1920x1080x500/rows0of2" "--shard 0/2"
add c2_r0of4 "random_spheres:1920x1080x500/rows0of4" "--shard 0/4"
add c2_r0of8 "random_spheres:1920x1080x500/rows0of8" "--shard 0/8"
[ -n "$ONLY" ] && { for i in "${!NAMES[@]}"; do [[ " $ONLY " == *" ${NAMES[$i]} "* ]] || unset 'NAMES[i]'; done; }
rc=0
for i in "${!NAMES[@]}"; do
  n=${NAMES[$i]}; k=${KEYS[$i]}; a=${ARGS[$i]}
  cmd="python bench.py --steps 1 --warmup 0 --no-cpu --no-hash --no-verify $a"; mkdir -p "$OUT/$n"
  for pass in valu fetch write; do
    case $pass in valu) P="$PV";; fetch) P="FETCH_SIZE";; write) P="WRITE_SIZE";; esac
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $P -d "$OUT/$n/$pass" -o run --output-format csv -- $cmd \
        > "$OUT/$n/$pass.log" 2>&1 || { rc=$?; echo "$n $pass failed rc=$rc"; break 2; }
  done
  python scripts/pmc_valu.py "$OUT/$n/valu" "$OUT/valu_r$R.jsonl" --workload "$k" --renders 1 > "$OUT/$n/valu.json" && \
  python scripts/pmc_traffic.py "$OUT/$n" "$OUT/traffic_r$R.jsonl" --workload "$k" --renders 1 > "$OUT/$n/traffic.json" || \
      { rc=$?; echo "$n summary failed"; break; }
  echo "$n: $(cut -c1-160 "$OUT/$n/valu.json")"
done
cp "$OUT/valu_r$R.jsonl" "$OUT/traffic_r$R.jsonl" profiles/ 2>/dev/null
echo "profiles rc=$rc"
exit $rc
