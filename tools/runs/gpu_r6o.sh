#!/bin/bash
# Round 6: zstd sequence-stage timing bound -- the window loads from a fixed
# (always cached) address, every sequence run (wrong values, timing only) --
# beside the product build; kernel traces of CZ, one process per build.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r6o}; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -1 | cut -c1-250 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
for L in ${LIBS:-zstv3 zstfix}; do
  OKV_LIB=tools/ab/r5/lib_$L.so step trace_$L 300 rocprofv3 --kernel-trace --stats -d $O/trace_$L -o run --output-format csv -- python3 bench.py --config cz --steps 10 --warmup 2 --no-cpu --no-verify
done
echo "r6o done"
