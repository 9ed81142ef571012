#!/bin/bash
# Round 6: the grouped single-pass small-block decode (okv_group_kernel):
# GPU suite; CM A/B against the two-pass form (r6d); host-mode small batches
# point vs NO_POINT; C5 kernel traces r6 vs r6c (line cut).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r6g}; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -1 | cut -c1-250 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
for i in 1 2; do
  for L in r6d r6e; do
    OKV_LIB=tools/ab/r5/lib_dec$L.so step cm_${L}_$i 300 python3 bench.py --config cm --no-cpu --steps 10 --warmup 2
  done
done
step point_batch 300 python3 tools/point_batch_ab.py 300
for L in r6 r6c; do
  OKV_LIB=tools/ab/r5/lib_dec$L.so step trace_c5_$L 300 rocprofv3 --kernel-trace --stats -d $O/trace_c5_$L -o run --output-format csv -- python3 bench.py --config c5 --steps 20 --warmup 5 --no-cpu --no-verify --decode-inflight 1
done
echo "r6g done"
