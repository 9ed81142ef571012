#!/bin/bash
# Round 5: point kernel phases (lean walk) + GetRow latency; SQ counters of
# the encode kernels; the C4 HBM traffic passes (FETCH/WRITE + calibration).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5i; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -2 | cut -c1-400 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
step point_tests 300 $T tests/test_point_gpu.py -m gpu
step getrow 120 tools/getrow_bench 2000
step getrow_phases 120 tools/getrow_bench_ablate 500
grep config $O/getrow.log $O/getrow_phases.log
step sq_c4 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d $O/sq_c4 -o run -- python3 bench.py --config c4 --steps 2 --warmup 1 --no-cpu --c4-inflight 1
step pmc_c4 900 tools/pmc_run.sh r5i/pmc_c4 bench.py --config c4 --steps 3 --warmup 1 --no-cpu --c4-inflight 1
echo "r5i done"
