#!/bin/bash
# Round 6: the big-block kernel after pass 3 and the chain event (late) vs
# ahead of the chain wait (early): decode tests, C5 / C3 lines alternating,
# the in-flight kernel trace of C5 with the late form.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r6k}; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -1 | cut -c1-250 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step tests 600 python -u -m pytest tests/test_decode_gpu.py tests/test_tile_gpu.py tests/test_bench_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread
for i in 1 2; do
  for L in early late; do
    OKV_LIB=tools/ab/r5/lib_dec$L.so step c5_${L}_$i 200 python3 bench.py --config c5 --no-cpu --no-verify --steps 40 --warmup 5
    OKV_LIB=tools/ab/r5/lib_dec$L.so step c3_${L}_$i 300 python3 bench.py --config c3 --no-cpu --no-verify --steps 20 --warmup 5
  done
done
step trace_c5_if 300 rocprofv3 --kernel-trace -d $O/trace_c5_if -o run --output-format csv -- python3 bench.py --config c5 --steps 40 --warmup 5 --no-cpu --no-verify
echo "r6k done"
