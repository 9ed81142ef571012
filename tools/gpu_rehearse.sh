#!/bin/bash
# 2-rank rehearsal of the multi-GPU bench on ONE GPU: both ranks map to device 0
# (--device-mod 1), control plane over gloo, 127.0.0.1 rendezvous.  Logs go to
# profiles/<round>/rehearse_2ranks_1gpu_gloo_<config>.log (world_size 2 and every
# rank's verify line are in each).
#   tools/gpu_rehearse.sh <round dir, e.g. r4> [configs...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
D=profiles/${1:-r4}
shift
mkdir -p "$D"
P=29517
for c in ${*:-c3 c5 c4}; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $P bench.py --gpus 2 --steps 5 --warmup 1 \
    --device-mod 1 --dist-backend gloo --config "$c" > "$D/rehearse_2ranks_1gpu_gloo_$c.log" 2>&1
  rc=$?
  echo "[rehearse $c] exit $rc"
  grep -E '^\[rank|"world_size"' "$D/rehearse_2ranks_1gpu_gloo_$c.log" | cut -c1-200 | tail -6
  [ $rc -ne 0 ] && exit $rc
  P=$((P + 1))
done
echo rehearse done
