#!/bin/bash
# Round 6: CM with the grouped single pass at 16 / 8 / 4 blocks per workgroup
# against the two-pass form (r6d); the encode pack kernel with and without
# its block hashes (ablation OKV_ENC_VARIANT 7 / 4).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r6h}; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -1 | cut -c1-250 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
for i in 1 2; do
  for L in r6d g16 g8 g4; do
    OKV_LIB=tools/ab/r5/lib_dec$L.so step cm_${L}_$i 300 python3 bench.py --config cm --no-cpu --steps 10 --warmup 2
  done
done
step enc_hash 600 python3 tools/ablate_enc.py --variants 7,4 --images 16384 --reps 5
echo "r6h done"
