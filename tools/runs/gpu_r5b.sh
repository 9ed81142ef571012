#!/bin/bash
# Round 5: point path + bloom tests, C++ GetRow latency, then the count-arrival
# A/B and the 64 KiB tile forms (tools/gpu_r5a.sh).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5b; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_point_gpu.py tests/test_reader_gpu.py tests/test_decode_gpu.py tests/test_encode_gpu.py -m gpu > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_zstd_gpu.py -m gpu > $O/zstd_product.log 2>&1
rc=$?; echo "zstd suite, product library (seq_table inlined): $(tail -1 $O/zstd_product.log)"; [ $rc -ne 0 ] && exit $rc
OKV_ABLATE=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_zstd_gpu.py -m gpu > $O/zstd_ztrace.log 2>&1
rc=$?; echo "zstd suite, ZTRACE ablation library (recorder in): $(tail -1 $O/zstd_ztrace.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 tools/getrow_bench 2000 > $O/getrow.log 2>&1
rc=$?; cat $O/getrow.log; [ $rc -ne 0 ] && exit $rc
echo "r5b done"
