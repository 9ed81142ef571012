#!/bin/bash
# Round 4: A/B measurements after the parity suites pass.
#   1. C3 decode: two pieces (default) vs one (OKV_OPEN_NO_PIECES), alternating processes
#   2. CZ decode: the executor at 1 dword / 4 groups / 5-wave cap (product) vs the round-3 form
#   3. C4 encode bench (single-pass plan, meta entries in the pack kernel) and the C3 bench
# Every step has its own time limit; the first failure ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
T=${1:-r4b}; O=gpurun_out/$T; mkdir -p $O
step() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$n] exit $rc"; tail -2 $O/$n.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc; return 0; }
LIB=objectkv_amd/libokv_sst.so
for r in 1 2 3; do
  ABL_FLAGS=0 step "ab_c3_pieces_$r" 200 python3 tools/ab_lib.py $LIB pieces
  ABL_FLAGS=4 step "ab_c3_onepiece_$r" 200 python3 tools/ab_lib.py $LIB one_piece
done
for r in 1 2; do
  step "ab_cz_new_$r" 200 python3 tools/ab_cz.py $LIB exec_1dw_4g_cap5
  step "ab_cz_old_$r" 200 python3 tools/ab_cz.py tools/ab/libokv_zold.so exec_2dw_8g
done
step bench_c4 400 python3 bench.py --config c4 --no-cpu
step bench_c3 400 python3 bench.py --config c3 --no-cpu
echo r4b done
