#!/bin/bash
# Round 6: the executor's match sources by t mod offset (lib_zstmod) vs the
# product: the zstd suite through the variant (OKV_LIB), then CZ traces.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r6zj}; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -1 | cut -c1-250 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
OKV_LIB=tools/ab/r5/lib_${VAR:-zstmod}.so step tests_var 400 python -u -m pytest tests/test_zstd_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread
for r in 1 2; do
  for L in ${BASE:-zstd5} ${VAR:-zstmod}; do
    OKV_LIB=tools/ab/r5/lib_$L.so step trace_${L}_$r 300 rocprofv3 --kernel-trace --stats -d $O/trace_${L}_$r -o run --output-format csv -- python3 bench.py --config cz --steps 10 --warmup 2 --no-cpu --no-verify
  done
done
echo "r6zj done"
