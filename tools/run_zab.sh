#!/bin/bash
# zstd executor A/B: zstd + GPU suites on the product build, then the zstd stage profile of
# each library build given (alternating, one process per run), then the CZ bench.
#   tools/run_zab.sh <tag> <lib>...
# Each step has its own time limit; the first failure ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
T=$1; shift; O=gpurun_out/$T; mkdir -p $O
step() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$n] exit $rc"; tail -3 $O/$n.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest_zstd 300 python3 -u -m pytest tests/test_zstd_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread
for r in 1 2; do
  for L in "$@"; do
    ZP_LIB=$L step "prof_$(basename $L .so)_$r" 200 python3 tools/zstd_prof.py 16384
  done
done
step bench_cz 300 python3 bench.py --config cz --no-cpu
[ -n "$FULL" ] && step pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
echo zab done
