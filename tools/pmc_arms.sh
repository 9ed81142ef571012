#!/bin/bash
# One L2-traffic counter pass (read/write requests, L2 hits/misses) per
# ablation arm of tools/ablate.py (run on the GPU box via gpurun).
#   tools/pmc_arms.sh <tag> <arm> [<arm> ...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
TAG=$1
shift
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
for A in "$@"; do
  D="$OUT/$(echo "$A" | tr ':' '_')"
  ABL_ROUNDS=1 timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum \
    --kernel-trace --output-format csv -d "$D" -o run -- python3 "$R/tools/ablate.py" "$A" > "$D.log" 2>&1
  rc=$?; echo "[$A] exit $rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
