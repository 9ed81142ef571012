#!/bin/bash
# HBM traffic passes (run on the GPU box via gpurun): rocprofv3 --pmc
# FETCH_SIZE and --pmc WRITE_SIZE in separate runs (TCC slots), kernel trace
# only, over any python command; then the 4 GiB calibration kernels of
# tools/copybw3 cal (known byte counts).  Summarise with tools/pmc_summary.py.
#   tools/pmc_run.sh <tag> <python args...>
#   e.g. tools/pmc_run.sh r2_pmc bench.py --steps 3 --warmup 1 --no-cpu
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
TAG=$1
shift
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/$C" -o run \
    -- python3 "$@" > "$OUT/$C.log" 2>&1
  rc=$?; echo "[$C] exit $rc"; [ $rc -ne 0 ] && exit $rc
done
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/cal_${C%%_SIZE}" -o run \
    -- "$R/tools/copybw3" cal > "$OUT/cal_$C.log" 2>&1
  rc=$?; echo "[cal $C] exit $rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
