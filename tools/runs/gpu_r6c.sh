#!/bin/bash
# Round 6: the sector-complete tile pass (ablation form d160) and the
# line-cut form (d96): parity through the tile / decode / full-size tests with
# the arm selected, PMC traffic and times against the product form; then the
# C5 in-flight / chaining grid (tools/runs/gpu_r6b.sh).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r6c}; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -1 | cut -c1-250 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
OKV_ABLATE=1 OKV_VALUE_SWEEP=8 OKV_TILE=16xd160 step tests_d160 600 python -u -m pytest tests/test_tile_gpu.py tests/test_decode_gpu.py tests/test_full_size_gpu.py::test_c3_full_decode_vs_oracle -m gpu -x -v --timeout 300 --timeout-method thread
ARMS="8:16x 8:16xd160 8:16xd96"
export ABL_ROUNDS=1 ABL_STEPS=2 ABL_CLASSES=1
for C in FETCH_SIZE WRITE_SIZE; do
  step pmc_$C 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/pmc_$C -o run -- python3 tools/ablate_tile.py $ARMS
done
export ABL_ROUNDS=7 ABL_STEPS=10
step time_arms 300 python3 tools/ablate_tile.py $ARMS
step time_arms2 300 python3 tools/ablate_tile.py 8:16xd160 8:16x
echo "r6c done"
