#!/bin/bash
# End-of-round-6 evidence at the committed sources (run on the GPU box via
# gpurun; everything lands under gpurun_out/<tag>/, copied into profiles/r6 by
# tools/runs/collect_r6.sh afterwards).  Two parts, each within one gpurun call:
#   a: GPU suite + smoke (as the driver runs them), C3 / C4 PMC passes
#      (FETCH_SIZE / WRITE_SIZE + 4 GiB calibration), the driver's bench
#      command (C3 with its CPU baseline), the C3 kernel trace one decode at a
#      time summarised against the traced process's own event time
#   b: the other configurations' bench lines (with CPU baselines), the CZ
#      kernel trace, GetRow latency, bimodal blocks, 2-rank one-GPU rehearsals
# Every step has its own time limit; the first failure ends the script.
#   tools/runs/gpu_final6.sh <a|b|b2> <tag>   (b2: b plus the driver's bench command)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
PART=${1:-a}
T=${2:-r6fin}
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
DSHA=$(python3 -c "import bench; print(bench.source_sha(bench.DECODE_SOURCES))")
ESHA=$(python3 -c "import bench; print(bench.source_sha(bench.ENCODE_SOURCES))")
ZSHA=$(python3 -c "import bench; print(bench.source_sha(bench.ZSTD_SOURCES))")
if [ "$PART" = a ]; then
  step pytest 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
  step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
  step pmc_c3 600 "$R/tools/pmc_run.sh" "$T/pmc_c3" bench.py --config c3 --steps 3 --warmup 1 \
    --no-cpu --no-verify --decode-inflight 1
  step pmc_c3_sum 60 python3 tools/pmc_summary.py "$O/pmc_c3" "$O/pmc_c3_full.json" \
    "{\"source_sha\": \"$DSHA\", \"config\": \"c3\", \"mode\": \"full\", \"source\": \"gpurun_out/$T/pmc_c3\"}"
  step pmc_c4 600 "$R/tools/pmc_run.sh" "$T/pmc_c4" bench.py --config c4 --steps 3 --warmup 1 \
    --no-cpu --no-verify --c4-inflight 1
  step pmc_c4_sum 60 python3 tools/pmc_summary.py "$O/pmc_c4" "$O/pmc_c4_encode.json" \
    "{\"source_sha\": \"$ESHA\", \"config\": \"c4\", \"mode\": \"encode\", \"source\": \"gpurun_out/$T/pmc_c4\"}"
  mkdir -p profiles/r6 && cp "$O/pmc_c3_full.json" "$O/pmc_c4_encode.json" profiles/r6/
  step trace_c3 300 rocprofv3 --kernel-trace --stats -d "$O/trace_c3" -o run --output-format csv \
    -- python3 "$R/bench.py" --config c3 --steps 20 --warmup 5 --no-cpu --no-verify --decode-inflight 1
  CSV=$(find "$O/trace_c3" -name 'run_kernel_trace.csv' | head -1)
  ALG=$(python3 -c "import json; l=[json.loads(x) for x in open('$O/trace_c3.log') if x.startswith('{')][-1]; print(l['roofline']['algorithmic_bytes_per_launch'])")
  step trace_c3_sum 60 python3 tools/trace_summary.py "$CSV" okv_tile_kernel 6 "$ALG" "$O/trace_c3.json" \
    "C3 one decode at a time (bench.py --decode-inflight 1, 20 steps + 5 warmup + guard)" \
    --sha "$DSHA" --bench-log "$O/trace_c3.log"
  cp "$O/trace_c3.json" profiles/r6/
  step bench_driver 600 python3 bench.py --gpus 1 --steps 20 --warmup 5
  echo "final6 a done"
else
  [ "$PART" = b2 ] && step bench_driver 600 python3 bench.py --gpus 1 --steps 20 --warmup 5
  if [ -n "$ENC_AGAIN" ]; then  # encode sources changed after part a: tests + C4 PMC again
    step enc_tests 600 python -u -m pytest tests/test_encode_gpu.py tests/test_snapshot_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread
    step pmc_c4 600 "$R/tools/pmc_run.sh" "$T/pmc_c4" bench.py --config c4 --steps 3 --warmup 1 \
      --no-cpu --no-verify --c4-inflight 1
    step pmc_c4_sum 60 python3 tools/pmc_summary.py "$O/pmc_c4" "$O/pmc_c4_encode.json" \
      "{\"source_sha\": \"$ESHA\", \"config\": \"c4\", \"mode\": \"encode\", \"source\": \"gpurun_out/$T/pmc_c4\"}"
    mkdir -p profiles/r6 && cp "$O/pmc_c4_encode.json" profiles/r6/
  fi
  step bench_c4 600 python3 bench.py --config c4
  # the zstd stage: its 9 kernels per decode summed (cap, prologue, seq offsets, streams,
  # sequences, executor, general, regrow list, descriptors); untimed: plan, guard, 2 warmup
  step trace_cz 300 rocprofv3 --kernel-trace --stats -d "$O/trace_cz" -o run --output-format csv \
    -- python3 "$R/bench.py" --config cz --steps 10 --warmup 2 --no-cpu --no-verify --decode-inflight 1
  CSV=$(find "$O/trace_cz" -name 'run_kernel_trace.csv' | head -1)
  ALG=$(python3 -c "import json; l=[json.loads(x) for x in open('$O/trace_cz.log') if x.startswith('{')][-1]; print(l['roofline']['algorithmic_bytes_per_launch'])")
  step trace_cz_sum 60 python3 tools/trace_summary.py "$CSV" okv_zstd_ 4 "$ALG" "$O/trace_cz.json" \
    "CZ one decode at a time (bench.py --decode-inflight 1, 10 steps + 2 warmup + guard + plan); the zstd stage's 9 kernels summed per decode" \
    --sha "$ZSHA" --bench-log "$O/trace_cz.log" --per-step 9 --event-key zstd
  mkdir -p profiles/r6 && cp "$O/trace_cz.json" profiles/r6/
  step bench_cz 600 python3 bench.py --config cz
  step bench_cm 600 python3 bench.py --config cm
  step trace_c5 300 rocprofv3 --kernel-trace --stats -d "$O/trace_c5" -o run --output-format csv \
    -- python3 "$R/bench.py" --config c5 --steps 20 --warmup 5 --no-cpu --no-verify --decode-inflight 1
  CSV=$(find "$O/trace_c5" -name 'run_kernel_trace.csv' | head -1)
  ALG=$(python3 -c "import json; l=[json.loads(x) for x in open('$O/trace_c5.log') if x.startswith('{')][-1]; print(l['roofline']['algorithmic_bytes_per_launch'])")
  step trace_c5_sum 60 python3 tools/trace_summary.py "$CSV" okv_tile_kernel 6 "$ALG" "$O/trace_c5.json" \
    "C5 one decode at a time (bench.py --decode-inflight 1, 20 steps + 5 warmup + guard)" \
    --sha "$DSHA" --bench-log "$O/trace_c5.log"
  mkdir -p profiles/r6 && cp "$O/trace_c5.json" profiles/r6/
  step bench_c5 300 python3 bench.py --config c5
  step bench_c2 300 python3 bench.py --config c2 --no-cpu
  step bench_c1 300 python3 bench.py --config c1 --no-cpu
  step getrow_latency 300 tools/getrow_bench 2000
  step getrow_phases 300 tools/getrow_bench_ablate 500
  step bench_e2e 600 python3 bench.py --e2e
  step mixed_blocks 300 python3 tools/mixed_blocks.py
  P=29517
  for c in c3 c5 c4; do
    step rehearse_2ranks_1gpu_gloo_$c 400 python3 -m torch.distributed.run --nnodes=1 \
      --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $P bench.py --gpus 2 --steps 5 \
      --warmup 1 --device-mod 1 --dist-backend gloo --config $c
    P=$((P + 1))
  done
  echo "final6 b done"
fi
