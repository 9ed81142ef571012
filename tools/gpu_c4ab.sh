#!/bin/bash
# C4 encode arms (ablation build): single-pass plan vs the E1-E9 kernels, meta
# entries fused into the pack kernel vs the separate meta kernel; the product last.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-c4ab}; mkdir -p $O
run() { local n=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-verify --steps 10 --warmup 3 > $O/$n.log 2>&1; local rc=$?;
  echo "[$n] exit $rc $(grep -o '"device_only_ms_per_step": [0-9.]*\|"kernel_ms": {[^}]*}' $O/$n.log | tr '\n' ' ')"; [ $rc -ne 0 ] && exit $rc; return 0; }
run fast_unfused OKV_ABLATE=1
run general_unfused OKV_ABLATE=1 OKV_ENC_GENERAL=1
run fast_fused OKV_ABLATE=1 OKV_ENC_META_FUSED=1
run general_fused OKV_ABLATE=1 OKV_ENC_GENERAL=1 OKV_ENC_META_FUSED=1
run product OKV_ABLATE=0
echo c4ab done
