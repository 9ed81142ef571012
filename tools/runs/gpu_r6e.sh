#!/bin/bash
# Round 6: GPU suite at the product sources (line-cut value ranges, the
# big-block kernel ahead of the chain wait); A/B of the bench lines C3 / C5
# against r6 (previous decode sources) alternating; C3 PMC traffic.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r6e}; mkdir -p $O
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
  for L in r6 r6c; do
    OKV_LIB=tools/ab/r5/lib_dec$L.so step c5_${L}_$i 200 python3 bench.py --config c5 --no-cpu --no-verify --steps 40 --warmup 5
    OKV_LIB=tools/ab/r5/lib_dec$L.so step c3_${L}_$i 300 python3 bench.py --config c3 --no-cpu --no-verify --steps 20 --warmup 5
  done
done
step pmc_c3 600 "$R/tools/pmc_run.sh" "${AB_TAG:-r6e}/pmc_c3" bench.py --config c3 --steps 3 --warmup 1 --no-cpu --no-verify --decode-inflight 1
echo "r6e done"
