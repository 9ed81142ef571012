#!/bin/bash
# zstd variants (product builds): the whole zstd suite, then a CZ kernel trace, per library
#   tools/gpu_zvar2.sh lib1.so [lib2.so ...]   (product = the in-tree build, first)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/zvar2; mkdir -p $O
cp objectkv_amd/libokv_sst.so /tmp/okv_product.so
for L in product "$@"; do
  if [ "$L" = product ]; then cp /tmp/okv_product.so objectkv_amd/libokv_sst.so; else cp "$L" objectkv_amd/libokv_sst.so; fi
  n=$(basename "$L" .so)
  timeout -k 10 300 python -u -m pytest tests/test_zstd_gpu.py -m gpu -q --timeout 200 > $O/t_$n.log 2>&1
  rc=$?; echo "[$n] tests exit $rc: $(tail -1 $O/t_$n.log)"; [ $rc -gt 1 ] && exit $rc
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr_$n -o run --output-format csv \
    -- python3 "$R/bench.py" --config cz --steps 10 --warmup 2 --no-cpu --no-verify --decode-inflight 1 > $O/b_$n.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "[$n] trace exit $rc"; exit $rc; }
  f=$(find $O/tr_$n -name run_kernel_stats.csv | head -1)
  echo "[$n] $(grep -h 'huf_kernel\|pro_kernel' $f | cut -d, -f1-4 | tr '\n' ' ') | $(grep -o '"zstd": [0-9.]*' $O/b_$n.log)"
done
exit 0
