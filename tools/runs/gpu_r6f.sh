#!/bin/bash
# Round 6: point path completion word (host spin instead of
# hipStreamSynchronize): reader / point / decode tests, GetRow latency A/B
# (tools/getrow_bench at the current sources vs r6c), host-mode small batches
# point vs NO_POINT, C5 kernel traces r6 vs r6c (line cut).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r6f}; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -1 | cut -c1-250 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step tests 600 python -u -m pytest tests/test_point_gpu.py tests/test_reader_gpu.py tests/test_decode_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread
for i in 1 2; do
  step getrow_new_$i 200 tools/getrow_bench 2000
  step getrow_r6c_$i 200 tools/ab/getrow_bench_r6c 2000
done
step point_batch 300 python3 tools/point_batch_ab.py 300
for L in r6 r6c; do
  OKV_LIB=tools/ab/r5/lib_dec$L.so step trace_c5_$L 300 rocprofv3 --kernel-trace --stats -d $O/trace_c5_$L -o run --output-format csv -- python3 bench.py --config c5 --steps 20 --warmup 5 --no-cpu --no-verify --decode-inflight 1
done
echo "r6f done"
