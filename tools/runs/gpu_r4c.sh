#!/bin/bash
# Product forms after the A/B: encode + decode GPU tests, then the bench lines.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
T=${1:-r4c}; O=gpurun_out/$T; mkdir -p $O
step() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$n] exit $rc"; tail -2 $O/$n.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc; return 0; }
step tests 600 python -u -m pytest tests/test_encode_gpu.py tests/test_decode_gpu.py tests/test_reader_gpu.py -m gpu -q --timeout 300 --timeout-method thread
step bench_c4 400 python3 bench.py --config c4 --no-cpu
step bench_c3 400 python3 bench.py --config c3 --no-cpu
step bench_cm 400 python3 bench.py --config cm --no-cpu
step bench_cz 400 python3 bench.py --config cz --no-cpu
step bench_c2 300 python3 bench.py --config c2 --no-cpu
echo r4c done
