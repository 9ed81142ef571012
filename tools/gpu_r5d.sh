#!/bin/bash
# Round 5 (one call): encode tests after the tile cut, the zstd suite
# (seq_table inlined), C++ GetRow latency, the C4 line, the per-block decode
# arms' parity and A/B against the tile pass, the count-arrival A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5d; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -2 | cut -c1-400 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step enc_tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_encode_gpu.py -m gpu
step zstd_product 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_zstd_gpu.py -m gpu
step getrow 120 tools/getrow_bench 2000
cat $O/getrow.log
step bench_c4 400 python3 bench.py --config c4 --steps 10 --warmup 3 --no-cpu
step check_block 300 env OKV_ABLATE=1 python3 tools/ablate_check.py block
step block_ab 400 env OKV_ABLATE=1 ABL_ROUNDS=4 python3 tools/ablate_tile.py 8:16x 9 10 11
cat $O/block_ab.log | tail -6
for r in 1 2; do
  for L in release relaxed; do
    step ab_count_${L}_$r 200 python3 tools/ab_lib.py tools/ab/r5/lib_$L.so $L
  done
done
echo "r5d done"
