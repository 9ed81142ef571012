#!/bin/bash
# PMC passes for the decode kernels (run on the GPU box via gpurun).
# Separate passes for FETCH_SIZE and WRITE_SIZE (TCC slots), kernel-trace only.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
TAG=${1:-pmc}
MODE=${2:-full}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/$C" -o run \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu --mode "$MODE" > "$OUT/$C.log" 2>&1
  rc=$?; echo "[$C] exit $rc"; [ $rc -ne 0 ] && exit $rc
done
# calibration on known byte counts (4 GiB copy / read / fill)
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/cal_FETCH" -o run \
  -- "$R/tools/copybw" > "$OUT/cal_FETCH.log" 2>&1; echo "[cal FETCH] exit $?"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/cal_WRITE" -o run \
  -- "$R/tools/copybw" > "$OUT/cal_WRITE.log" 2>&1; echo "[cal WRITE] exit $?"
find "$OUT" -name '*counter_collection*' | head
