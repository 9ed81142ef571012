#!/bin/bash
# C4 pack-kernel arms: tools/c4_arms.sh "VAR:IMG" ...  (OKV_ENC_VARIANT, OKV_ENC_IMAGE)
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for arm in "$@"; do
  v=${arm%%:*}; img=${arm##*:}
  echo "== arm variant=$v image=$img"
  OKV_ENC_VARIANT=$v OKV_ENC_IMAGE=$img timeout -k 10 150 python3 -u bench.py --config c4 --steps 10 --warmup 3 \
    --c4-inflight 1 --no-verify > gpurun_out/c4arm.log 2>&1 || exit $?
  python3 -c "import json,sys; l=[x for x in open('gpurun_out/c4arm.log') if x.startswith('{')][-1]; d=json.loads(l); print(d['kernel_ms'], d['device_only_ms_per_step'])"
done
