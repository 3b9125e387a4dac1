#!/bin/bash
# gpurun: PMC counter passes (one rocprofv3 run per pass, --pmc only with kernel trace)
# over a short render.  Output: gpurun_out/$PMC_TAG/<pass>/..._counter_collection.csv
#   PMC_CMD  the program to profile (default: the headline bench, one timed step)
#   PMC_TAG  output directory under gpurun_out (default pmc)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${PMC_TAG:-pmc}
OUT="$PWD/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp
CMD=${PMC_CMD:-"python bench.py --steps 1 --warmup 0 --no-cpu --no-verify"}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
P2="SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
P5="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
i=0; rc=0
for P in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE" "$P5"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $P -d "$OUT/p$i" -o run --output-format csv -- $CMD > "$OUT/p$i.log" 2>&1 || { rc=$?; break; }
  echo "pass $i done"
done
echo "exit=$rc"
exit $rc
