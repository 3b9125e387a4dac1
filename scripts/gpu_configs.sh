#!/bin/bash
# gpurun: one bench line per config and demo scene on this library, each with its
# roofline from profiles/{valu,traffic}_r$ROUND.jsonl (scripts/gpu_profiles.sh, same library by hash), the
# CPU oracle timed beside the small ones (10-20 steps for the ones of a few ms); a rocprofv3 kernel trace of the
# Cornell box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${ROUND:-06}; OUT="$PWD/gpurun_out/${TAG:-configs$R}"; mkdir -p "$OUT"; export TMPDIR=/tmp
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python bench.py --steps 3 --warmup 1 --cpu-target-s 5 --valu profiles/valu_r$R.jsonl --traffic profiles/traffic_r$R.jsonl "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" || return $?
  tail -1 "$OUT/$n.json" >> "$OUT/configs.jsonl"
  tail -1 "$OUT/$n.json" | cut -c1-220
}
: > "$OUT/configs.jsonl"
run c2_random_spheres_1920 --no-cpu && \
run c1_random_spheres_400 --width 400 --spp 100 --steps 20 --warmup 3 && \
run c3_random_spheres_2000 --spp 2000 --no-cpu && \
run c4_stress_100k --scene stress_100k --spp 100 && \
run c5_earth_dielectric --scene earth_dielectric --width 3840 --spp 1000 --no-cpu && \
run cornell_box --scene cornell_box --width 600 --spp 200 --steps 10 --warmup 2 && \
run quad_demo --scene quad_demo --width 400 --spp 100 --steps 20 --warmup 3 && \
run perlin_demo --scene perlin_demo --width 400 --spp 100 --steps 20 --warmup 3 && \
run simple_light_demo --scene simple_light_demo --width 400 --spp 500 --steps 10 --warmup 2 && \
for n in 2 4 8; do run c2_shard0of$n --shard 0/$n --no-cpu || exit $?; done && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_cornell" -o run --output-format csv -- \
    python bench.py --scene cornell_box --width 600 --spp 200 --steps 2 --warmup 1 --no-cpu > "$OUT/cornell_prof.log" 2>&1
rc=$?
echo "configs rc=$rc"
exit $rc
