#!/bin/bash
# zstd variant check on the box's copy of the tree: each named library in turn
# replaces objectkv_amd/libokv_sst.so for one pytest selection.
#   tools/gpu_zvar.sh "<pytest -k expr>" lib1.so [lib2.so ...]   (product = the in-tree build)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
mkdir -p gpurun_out
K=$1; shift
cp objectkv_amd/libokv_sst.so /tmp/okv_product.so
for L in product "$@"; do
  if [ "$L" = product ]; then cp /tmp/okv_product.so objectkv_amd/libokv_sst.so; else cp "$L" objectkv_amd/libokv_sst.so; fi
  n=$(basename "$L" .so)
  timeout -k 10 240 python -u -m pytest tests/test_zstd_gpu.py -k "$K" -q --timeout 200 > gpurun_out/zvar_$n.log 2>&1
  rc=$?
  echo "[$n] exit $rc: $(tail -1 gpurun_out/zvar_$n.log)"
  [ $rc -gt 1 ] && exit $rc
done
exit 0
