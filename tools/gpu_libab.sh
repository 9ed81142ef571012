#!/bin/bash
# A/B of product libraries on one box: each library in turn replaces
# objectkv_amd/libokv_sst.so; the first one also runs the given test files.
#   tools/gpu_libab.sh "<tests>" "<bench args>" <rounds> lib1.so lib2.so ...
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/libab; mkdir -p $O
TESTS=$1; BARGS=$2; ROUNDS=$3; shift 3
cp "$1" objectkv_amd/libokv_sst.so
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "[tests $(basename $1)] exit $rc: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && exit $rc
fi
for r in $(seq 1 $ROUNDS); do
  for L in "$@"; do
    cp "$L" objectkv_amd/libokv_sst.so
    n=$(basename "$L" .so)
    timeout -k 10 300 python3 bench.py $BARGS > $O/${n}_$r.log 2>&1
    rc=$?; echo "[$n run $r] exit $rc $(grep -o '"value": [0-9.]*\|"stage_ms": {[^}]*}\|"kernel_ms": {[^}]*}\|"frac": [0-9.]*' $O/${n}_$r.log | head -4 | tr '\n' ' ')"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
