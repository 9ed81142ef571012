#!/bin/bash
# Encode-side evidence after an encode-only change (run on the GPU box via gpurun): the GPU
# suite + smoke, the C4 PMC passes (-> profiles/r4/pmc_c4_encode.json on the box), then the lines
# that run the encoder (C4 with the PMC attached, CM, C1) and the C4 2-rank rehearsal.
#   tools/gpu_final_enc.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
T=${1:-final9}
O="$R/gpurun_out/$T"
mkdir -p "$O"
step() {
  local n=$1 s=$2
  shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc"
  grep -v amdgpu.ids "$O/$n.log" | tail -2 | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
  return 0
}
ESHA=$(python3 -c "import bench; print(bench.source_sha(bench.ENCODE_SOURCES))")
step pytest 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step pmc_c4 600 "$R/tools/pmc_run.sh" "$T/pmc_c4" bench.py --config c4 --steps 3 --warmup 1 \
  --no-cpu --no-verify --c4-inflight 1
step pmc_c4_sum 60 python3 tools/pmc_summary.py "$O/pmc_c4" "$O/pmc_c4_encode.json" \
  "{\"source_sha\": \"$ESHA\", \"config\": \"c4\", \"mode\": \"encode\", \"source\": \"gpurun_out/$T/pmc_c4\"}"
mkdir -p profiles/r4 && cp "$O/pmc_c4_encode.json" profiles/r4/
step bench_c4 600 python3 bench.py --config c4
step bench_cm 600 python3 bench.py --config cm
step bench_c1 300 python3 bench.py --config c1 --no-cpu
step rehearse_2ranks_1gpu_gloo_c4 400 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 \
  --warmup 1 --device-mod 1 --dist-backend gloo --config c4
echo "final enc done"
exit 0
