#!/bin/bash
# Round 5: encode A/B of several builds on one box (tools/ab/r5/lib_enc<X>.so
# for X in $ARMS): encode tests against each arm, then the C4 line per arm,
# alternating, three rounds.  NOTEST: arms whose tests are skipped
# (diagnostic builds, e.g. no block hashes).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r5v}; mkdir -p $O
ARMS=${ARMS:-"A B"}
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -2 | cut -c1-300 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
for L in $ARMS; do
  case " $NOTEST " in *" $L "*) continue ;; esac  # diagnostic arms (wrong hashes by design)
  step enc_tests_$L 600 env OKV_LIB=tools/ab/r5/lib_enc$L.so $T tests/test_encode_gpu.py -m gpu
done
for r in 1 2 3; do
  for L in $ARMS; do
    step ab_${L}_$r 300 env OKV_LIB=tools/ab/r5/lib_enc$L.so python3 bench.py --config c4 --steps 10 --warmup 3 --no-cpu --no-verify
    echo "  $L $r: $(grep -o '"device_only_ms_per_step[^}]*}' $O/ab_${L}_$r.log)"
  done
done
echo "r5v done"
