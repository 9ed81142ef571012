#!/bin/bash
# Round 6: C5 (1 GiB segment, the per-GPU workload of the 8-GPU config) --
# decodes in flight 2 / 4, pass 3 chained or not, alternating; then the
# kernel trace of the C5 bench one decode at a time.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r6b}; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -1 | cut -c1-200 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
for i in 1 2; do
  for a in "2 on" "2 off" "4 on" "4 off" "1 auto"; do
    set -- $a
    step c5_if$1_$2_$i 200 python3 bench.py --config c5 --no-cpu --no-verify --steps 40 --warmup 5 --decode-inflight $1 --pass3-chain $2
  done
done
step trace_c5 300 rocprofv3 --kernel-trace --stats -d $O/trace_c5 -o run --output-format csv -- python3 bench.py --config c5 --steps 20 --warmup 5 --no-cpu --no-verify --decode-inflight 1
echo "r6b done"
