#!/bin/bash
# Round 6: the count kernel's record chunk (records per lane between LDS
# flushes) 16 (product) vs 8 (half its LDS: 7 tile workgroups fit beside it
# instead of 6): decode tests through the variant, then C3 / C5 / CM / C2 lines
# alternating, in-flight C5 traces.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r6ad}; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -1 | cut -c1-250 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
OKV_LIB=tools/ab/r5/lib_decrc8.so step tests_rc8 600 python -u -m pytest tests/test_decode_gpu.py tests/test_tile_gpu.py tests/test_reader_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread
for i in 1 2; do
  for L in rc16 rc8; do
    OKV_LIB=tools/ab/r5/lib_dec$L.so step c3_${L}_$i 300 python3 bench.py --config c3 --no-cpu --no-verify --steps 20 --warmup 5
    OKV_LIB=tools/ab/r5/lib_dec$L.so step c5_${L}_$i 200 python3 bench.py --config c5 --no-cpu --no-verify --steps 40 --warmup 5
    OKV_LIB=tools/ab/r5/lib_dec$L.so step cm_${L}_$i 300 python3 bench.py --config cm --no-cpu --no-verify --steps 10 --warmup 2
    OKV_LIB=tools/ab/r5/lib_dec$L.so step c2_${L}_$i 200 python3 bench.py --config c2 --no-cpu --no-verify --steps 40 --warmup 5
  done
done
echo "r6ad done"
