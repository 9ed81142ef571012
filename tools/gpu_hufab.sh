#!/bin/bash
# zstd stream stage: blocks per wave (ablation build, OKV_ZSTD_HUF_BLOCKS), CZ kernel trace per arm
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-hufab}; mkdir -p $O
for hb in 16 8 4 2; do
  OKV_ABLATE=1 OKV_ZSTD_HUF_BLOCKS=$hb timeout -k 10 400 python -u -m pytest tests/test_zstd_gpu.py -m gpu -q \
    -k "test_zstd_cases and staged" --timeout 300 --timeout-method thread > $O/tests_$hb.log 2>&1
  rc=$?; echo "[zstd cases, $hb blocks per wave] exit $rc: $(tail -1 $O/tests_$hb.log)"
done
for hb in 16 8 4 2; do
  OKV_ABLATE=1 OKV_ZSTD_HUF_BLOCKS=$hb timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t$hb -o run --output-format csv \
    -- python3 "$R/bench.py" --config cz --steps 10 --warmup 2 --no-cpu --no-verify --decode-inflight 1 > $O/hb_$hb.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "[hb $hb] exit $rc"; exit $rc; }
  f=$(find $O/t$hb -name run_kernel_stats.csv | head -1)
  echo "[hb $hb] $(grep -h huf_kernel $f | cut -d, -f1-4) | $(grep -o '"zstd": [0-9.]*' $O/hb_$hb.log)"
done
exit 0
