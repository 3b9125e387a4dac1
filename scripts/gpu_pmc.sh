#!/bin/bash
# gpurun: PMC counter passes (one rocprofv3 run per pass, --pmc only with kernel trace)
# over a short render.  Output: gpurun_out/pmc/<pass>/..._counter_collection.csv
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out"; mkdir -p "$OUT/pmc"; export TMPDIR=/tmp
CMD=${PMC_CMD:-"python scripts/ab.py --spp 50 --rounds 1 --variants v1"}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
P2="SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
i=0; rc=0
for P in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P -d "$OUT/pmc/p$i" -o run --output-format csv -- $CMD > "$OUT/pmc/p$i.log" 2>&1 || { rc=$?; break; }
done
echo "exit=$rc"; ls "$OUT/pmc"/*/ 2>/dev/null | head
exit $rc
