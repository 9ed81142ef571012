#!/bin/bash
# Round 6: the sequence stage's prefetch wave by lead (lib_zst<NAME>.so
# builds), CZ kernel traces, one process per build, two rounds.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r6s}; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -1 | cut -c1-250 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
[ -n "$TESTS" ] && step tests_zstd 400 python -u -m pytest tests/test_zstd_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread
for r in 1 2; do
  for L in ${LIBS:-zstv3 zstpf64 zstpf16 zstpf64b}; do
    OKV_LIB=tools/ab/r5/lib_$L.so step trace_${L}_$r 300 rocprofv3 --kernel-trace --stats -d $O/trace_${L}_$r -o run --output-format csv -- python3 bench.py --config cz --steps 10 --warmup 2 --no-cpu --no-verify
  done
done
echo "r6s done"
