#!/bin/bash
# Round 5: pack-kernel shapes on one box (ablation build): the product
# (16 KiB image, 256 threads: one wave hashes 4 blocks on 16 lanes) vs 32 KiB /
# 512 threads (8 blocks) vs 64 KiB / 1 024 threads (16 blocks, all 64 lanes).
# Round 1 of each arm checks the whole segment file against the oracle writer.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5q; mkdir -p $O
run() {  # name, round, env...
  local n=$1 r=$2; shift 2
  local v="--no-verify"; [ "$r" = 1 ] && v=""
  timeout -k 10 300 env OKV_ABLATE=1 "$@" python3 bench.py --config c4 --steps 10 --warmup 3 --no-cpu $v > $O/${n}_$r.log 2>&1
  local rc=$?
  echo "[$n $r] exit $rc $(grep -o 'whole segment file == oracle writer' $O/${n}_$r.log) $(grep -o '"device_only_ms_per_step[^}]*}' $O/${n}_$r.log)"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
for r in 1 2 3; do
  run img16k_256 $r OKV_ENC_NOTHING=0
  run img32k_512 $r OKV_ENC_IMAGE=32768 OKV_ENC_VARIANT=10
  run img64k_1024 $r OKV_ENC_IMAGE=65536
done
echo "r5q done"
