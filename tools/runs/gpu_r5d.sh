#!/bin/bash
# Round 5: decode A/B (tools/ab/r5/lib_decA.so = before, lib_decB.so = after):
# the GPU suite on the in-tree product build (= B), then CM and C3 lines
# alternating, three rounds each.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r5d}; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -2 | cut -c1-300 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
[ -z "$NOTESTS" ] && step tests 900 $T tests -m gpu
for r in 1 2 3; do
  for L in A B; do
    step cm_${L}_$r 300 env OKV_LIB=tools/ab/r5/lib_dec$L.so python3 bench.py --config cm --steps 10 --warmup 3 --no-cpu
    echo "  cm $L $r: $(grep -o '"stage_ms": {[^}]*}' $O/cm_${L}_$r.log)"
  done
done
for r in 1 2 3; do
  for L in A B; do
    step c3_${L}_$r 300 env OKV_LIB=tools/ab/r5/lib_dec$L.so python3 bench.py --steps 10 --warmup 3 --no-cpu
    echo "  c3 $L $r: $(grep -o '"ms_per_step": [0-9.]*' $O/c3_${L}_$r.log) $(grep -o '"latency_ms_per_step": [0-9.]*' $O/c3_${L}_$r.log) $(grep -o '"frac_pass3": [0-9.]*' $O/c3_${L}_$r.log)"
  done
done
echo "r5d done"
