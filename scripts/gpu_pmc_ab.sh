#!/bin/bash
# gpurun: PMC passes (VALU / SALU / LDS instructions; wave cycles and waits) of one render, tiered
# and not (scripts/render_once.py), under gpurun_out/$TAG/{tier,notier}/p*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-pmcab}; OUT="$PWD/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
P2="SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
for v in tier notier; do
  arg=""; [ $v = notier ] && arg="--no-tier"; mkdir -p "$OUT/$v"
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $P -d "$OUT/$v/p$i" -o run --output-format csv -- \
        python scripts/render_once.py --spp ${SPP:-100} $arg > "$OUT/$v/p$i.log" 2>&1 || { echo "pmc failed rc=$?"; exit 1; }
    echo "$v pass $i done"
  done
done
