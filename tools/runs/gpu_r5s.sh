#!/bin/bash
# Round 5: the wave-cooperative count walk for large segments of small blocks
# (okv_count_kernel<true>): decode / reader / snapshot tests, then the CM line
# A/B on one box (ablation build, OKV_COUNT_WAVE=0 / 1 alternating), a CM trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5s; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -2 | cut -c1-300 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
step dec_tests 900 $T tests/test_decode_gpu.py tests/test_tile_gpu.py tests/test_reader_gpu.py tests/test_snapshot_gpu.py -m gpu
for r in 1 2 3; do
  for wv in 0 1; do
    step cm_wave${wv}_$r 400 env OKV_ABLATE=1 OKV_COUNT_WAVE=$wv python3 bench.py --config cm --steps 10 --warmup 2 --no-cpu
    echo "  wave=$wv $r: $(grep -o '"stage_ms": {[^}]*}' $O/cm_wave${wv}_$r.log) $(grep -o '"value": [0-9.]*' $O/cm_wave${wv}_$r.log | head -1)"
  done
done
step trace_cm 300 rocprofv3 --kernel-trace --stats -d $O/trace_cm -o run -- python3 bench.py --config cm --steps 3 --warmup 1 --no-cpu
echo "r5s done"
