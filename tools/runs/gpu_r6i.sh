#!/bin/bash
# Round 6: the tile pass's per-lane key / boundary loop started on the last
# wave (bal) against wave 0 (nobal), C3 one decode at a time, alternating;
# C3 with four decodes in flight, pass 3 chained or not.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r6i}; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -1 | cut -c1-250 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
for i in 1 2 3; do
  for L in nobal bal; do
    ABL_ROUNDS=7 ABL_STEPS=10 step ab_c3_${L}_$i 200 python3 tools/ab_lib.py tools/ab/r5/lib_dec$L.so $L
  done
done
for i in 1 2; do
  for c in on off; do
    step c3_if4_${c}_$i 300 python3 bench.py --config c3 --no-cpu --no-verify --steps 20 --warmup 5 --pass3-chain $c
  done
done
echo "r6i done"
