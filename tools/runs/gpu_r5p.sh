#!/bin/bash
# Round 5: encode A/B of two builds on one box (tools/ab/r5/lib_encA.so vs lib_encB.so),
# entry-chain bound) -- tests, then an A/B of the two builds on one box
# (tools/ab/r5/lib_encA.so = before, lib_encB.so = after), C4 line alternating.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r5p}; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -2 | cut -c1-300 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
step enc_tests 600 $T tests/test_encode_gpu.py tests/test_snapshot_gpu.py -m gpu
for r in 1 2 3; do
  for L in A B; do
    step ab_${L}_$r 300 env OKV_LIB=tools/ab/r5/lib_enc$L.so python3 bench.py --config c4 --steps 10 --warmup 3 --no-cpu --no-verify
    echo "  $L $r: $(grep -o '"device_only_ms_per_step[^}]*}' $O/ab_${L}_$r.log)"
  done
done
step trace_c4 300 rocprofv3 --kernel-trace --stats -d $O/trace_c4 -o run -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu --c4-inflight 1 --no-verify
echo "r5p done"
