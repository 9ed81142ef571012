#!/bin/bash
# Round 6: the GPU suite at the current product sources (fused kernel with the
# LDS pre-assembly, chained decodes on a shared pass-3 stream); C2 A/B of the
# fused forms; the fused phases; C5 / C3 in-flight lines with the shared
# pass-3 stream (r6b) against the cross-stream event chain (r6); the sector
# form variants d672 / d928 against the product tile pass.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r6d}; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -1 | cut -c1-250 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
for i in 1 2 3; do
  for L in r6 r6b; do
    ABL_NBLK=256 ABL_KIND=0 ABL_BS=4096 ABL_TH=3584 ABL_ROUNDS=7 ABL_STEPS=50 \
      step ab_c2_${L}_$i 120 python3 tools/ab_lib.py tools/ab/r5/lib_dec$L.so $L
  done
done
step fused_phases 120 python3 tools/fused_phases.py
for i in 1 2; do
  for L in r6 r6b; do
    OKV_LIB=tools/ab/r5/lib_dec$L.so step c5_${L}_$i 200 python3 bench.py --config c5 --no-cpu --no-verify --steps 40 --warmup 5
  done
done
for i in 1 2; do
  for L in r6 r6b; do
    OKV_LIB=tools/ab/r5/lib_dec$L.so step c3_${L}_$i 300 python3 bench.py --config c3 --no-cpu --no-verify --steps 20 --warmup 5
  done
done
export ABL_ROUNDS=7 ABL_STEPS=10
step time_arms 300 python3 tools/ablate_tile.py 8:16x 8:16xd672 8:16xd928 8:16xd96
echo "r6d done"
