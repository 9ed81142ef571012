#!/bin/bash
# GPU suite, then bench lines (C3 chained in-flight + one at a time, C5, C2, CZ) and the zstd
# stage/prologue profile.  Each step has its own time limit; the first failure ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
T=${1:-r3f}; O=gpurun_out/$T; mkdir -p $O
step() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$n] exit $rc"; tail -2 $O/$n.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_c3 300 python3 bench.py --config c3 --no-cpu
step bench_c3_one 300 python3 bench.py --config c3 --no-cpu --no-verify --decode-inflight 1
step bench_c5 300 python3 bench.py --config c5 --no-cpu --no-verify
step bench_c2 300 python3 bench.py --config c2 --no-cpu --no-verify
step bench_cz 300 python3 bench.py --config cz --no-cpu --no-verify
OKV_ABLATE=1 step zstd_prof 300 python3 tools/zstd_prof.py 16384
OKV_ABLATE=1 step ablate_enc 400 python3 tools/ablate_enc.py --variants 7,4,5 --images 16384 --reps 3
echo r3f done
