#!/bin/bash
# gpurun: the non-headline configs of SURVEY §8(d) and the Cornell box, one bench line
# each (counts + roofline + CPU sample), plus a rocprofv3 kernel trace of the Cornell run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-configs}"; mkdir -p "$OUT"; export TMPDIR=/tmp
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python bench.py --steps 2 --warmup 1 --cpu-target-s 5 "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" || return $?
  tail -1 "$OUT/$n.json"
}
run c1_random_spheres_400 --width 400 --spp 100 && \
run c3_random_spheres_2000 --width 1920 --spp 2000 --no-cpu && \
run c4_stress_100k --scene stress_100k --width 1920 --spp 100 && \
RTX_BVH=guarded run c4_stress_100k_guarded --scene stress_100k --width 1920 --spp 100 --no-cpu && \
run c5_earth_dielectric --scene earth_dielectric --width 3840 --spp 1000 --no-cpu && \
run cornell_box --scene cornell_box --width 600 --spp 200 && \
run quad_demo --scene quad_demo --width 400 --spp 100 && \
run perlin_demo --scene perlin_demo --width 400 --spp 100 && \
run simple_light_demo --scene simple_light_demo --width 400 --spp 500 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_cornell" -o run --output-format csv -- \
    python bench.py --scene cornell_box --width 600 --spp 200 --steps 2 --warmup 1 --no-cpu > "$OUT/cornell_prof.log" 2>&1
rc=$?
echo "exit=$rc"
exit $rc
