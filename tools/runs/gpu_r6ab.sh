#!/bin/bash
# Round 6: C5 / C3 without the big-block kernel launch (timing bound; C3 / C5
# have no big blocks) beside the product: bench lines alternating, in-flight
# kernel traces of C5.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r6ab}; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -1 | cut -c1-250 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
for i in 1 2; do
  for L in ${LIBS:-head nobig}; do
    OKV_LIB=tools/ab/r5/lib_dec$L.so step c5_${L}_$i 200 python3 bench.py --config c5 --no-cpu --no-verify --steps 40 --warmup 5
    OKV_LIB=tools/ab/r5/lib_dec$L.so step c3_${L}_$i 300 python3 bench.py --config c3 --no-cpu --no-verify --steps 20 --warmup 5
  done
done
for L in ${LIBS:-head nobig}; do
  OKV_LIB=tools/ab/r5/lib_dec$L.so step trace_c5_$L 300 rocprofv3 --kernel-trace --stats -d $O/trace_c5_$L -o run --output-format csv -- python3 bench.py --config c5 --steps 40 --warmup 5 --no-cpu --no-verify
done
echo "r6ab done"
