#!/bin/bash
# Round 6: the zstd sequence stage without the value work (extra bits, repeat
# offsets moved to the executor's check pass): zstd GPU suite, CZ lines
# alternating with the previous build, kernel traces of both.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r6l}; mkdir -p $O
OLD=${OLD_LIB:-tools/ab/libokv_zr6.so}
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -1 | cut -c1-250 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step tests_zstd 400 python -u -m pytest tests/test_zstd_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread
for i in 1 2; do
  step cz_new_$i 200 python3 bench.py --config cz --no-cpu --no-verify --steps 20 --warmup 3
  OKV_LIB=$OLD step cz_old_$i 200 python3 bench.py --config cz --no-cpu --no-verify --steps 20 --warmup 3
done
step trace_new 300 rocprofv3 --kernel-trace --stats -d $O/trace_new -o run --output-format csv -- python3 bench.py --config cz --steps 10 --warmup 2 --no-cpu --no-verify
OKV_LIB=$OLD step trace_old 300 rocprofv3 --kernel-trace --stats -d $O/trace_old -o run --output-format csv -- python3 bench.py --config cz --steps 10 --warmup 2 --no-cpu --no-verify
[ -n "$FULL" ] && step tests_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
echo "r6l done"
