#!/bin/bash
# VGPR / spill / scratch of the megakernel instantiations in a built rtx_kernel.o (no GPU needed).
#   bash scripts/kernel_resources.sh [raytracer-go_amd/build/rtx_kernel.o] [kernel-name filter]
set -o pipefail
OBJ=$(realpath "${1:-raytracer-go_amd/build/rtx_kernel.o}"); PAT=${2:-render_items<false}
T=$(mktemp -d); trap 'rm -rf "$T"' EXIT
L=/opt/rocm/lib/llvm/bin
$L/llvm-objcopy --dump-section .hip_fatbin="$T/fat.bin" "$OBJ" && \
$L/clang-offload-bundler --unbundle --type=o --input="$T/fat.bin" --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$T/k.co" && \
$L/llvm-readelf --notes "$T/k.co" | c++filt | python3 -c '
import sys, re
pat = sys.argv[1]
cur = {}
rows = []
for line in sys.stdin:
    m = re.match(r"\s+\.(name|vgpr_count|vgpr_spill_count|sgpr_spill_count|private_segment_fixed_size|sgpr_count):\s+(.*)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "name":
        if cur.get("name"):
            rows.append(cur)
        cur = {"name": v}
    else:
        cur[k] = v
if cur.get("name"):
    rows.append(cur)
for r in rows:
    if pat in r["name"] and not r["name"].endswith(".kd"):
        print(r.get("vgpr_count"), r.get("vgpr_spill_count"), r.get("sgpr_count"), r.get("sgpr_spill_count"), r.get("private_segment_fixed_size"), r["name"])
' "$PAT"
