set -o pipefail
cd "${GRAFT_REPO_ROOT}"
OUT="$PWD/gpurun_out"; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  RTX_LIB=$PWD/abl/librtx_base.so timeout -k 10 200 python scripts/ab.py --spp 100 --rounds 3 --variants v3 > "$OUT/ab_base_$i.log" 2>&1 || exit 1
  timeout -k 10 200 python scripts/ab.py --spp 100 --rounds 3 --variants v3 > "$OUT/ab_new_$i.log" 2>&1 || exit 1
  head -1 "$OUT/ab_base_$i.log"; head -1 "$OUT/ab_new_$i.log"
done
