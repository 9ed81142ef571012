#!/bin/bash
# zstd + encode iteration: zstd suite, GPU suite, CZ bench, zstd stage profile, encode pack A/B
# (7 = product, 9 = hashes overlapped with the image stores).  Each step has its own time
# limit; the first failure ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
T=${1:-r3i}; O=gpurun_out/$T; mkdir -p $O
step() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$n] exit $rc"; tail -3 $O/$n.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest_zstd 300 python3 -u -m pytest tests/test_zstd_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread
step pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_cz 300 python3 bench.py --config cz --no-cpu
OKV_ABLATE=1 step zstd_prof 300 python3 tools/zstd_prof.py 16384
OKV_ABLATE=1 step ablate_enc 400 python3 tools/ablate_enc.py --variants 7,9 --images 16384 --reps 5
echo r3i done
