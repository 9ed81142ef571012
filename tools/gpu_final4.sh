#!/bin/bash
# End-of-round-4 evidence at the committed sources (run on the GPU box via gpurun):
#   1. C3 PMC passes (FETCH_SIZE / WRITE_SIZE + 4 GiB calibration) -> profiles/r4/pmc_c3_full.json
#      (decode sources' SHA: the bench attaches the traffic); C4 likewise -> pmc_c4_encode.json
#   2. the driver's bench command (C3, CPU baseline included)
#   3. the C3 kernel trace one decode at a time -> profiles/r4/trace_c3.json (two tile launches
#      per decode summed; the traced process's own event time beside it)
#   4. the other configurations' bench lines; CZ kernel trace
# Every step has its own time limit; the first failure ends the script.
#   tools/gpu_final4.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
T=${1:-final4}
O="$R/gpurun_out/$T"
mkdir -p "$O" profiles/r4
step() {
  local n=$1 s=$2
  shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc"
  tail -2 "$O/$n.log" | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
  return 0
}
DSHA=$(python3 -c "import bench; print(bench.source_sha(bench.DECODE_SOURCES))")
ESHA=$(python3 -c "import bench; print(bench.source_sha(bench.ENCODE_SOURCES))")
step pmc_c3 600 "$R/tools/pmc_run.sh" "$T/pmc_c3" bench.py --config c3 --steps 3 --warmup 1 \
  --no-cpu --no-verify --decode-inflight 1
step pmc_c3_sum 60 python3 tools/pmc_summary.py "$O/pmc_c3" "$O/pmc_c3_full.json" \
  "{\"source_sha\": \"$DSHA\", \"config\": \"c3\", \"mode\": \"full\", \"source\": \"gpurun_out/$T/pmc_c3\", \"launches_per_step\": {\"okv_tile_kernel\": 2, \"okv_count_kernel\": 2}}"
step pmc_c4 600 "$R/tools/pmc_run.sh" "$T/pmc_c4" bench.py --config c4 --steps 3 --warmup 1 \
  --no-cpu --no-verify --c4-inflight 1
step pmc_c4_sum 60 python3 tools/pmc_summary.py "$O/pmc_c4" "$O/pmc_c4_encode.json" \
  "{\"source_sha\": \"$ESHA\", \"config\": \"c4\", \"mode\": \"encode\", \"source\": \"gpurun_out/$T/pmc_c4\"}"
cp "$O/pmc_c3_full.json" "$O/pmc_c4_encode.json" profiles/r4/
step bench_driver 600 python3 bench.py --gpus 1 --steps 20 --warmup 5
step trace_c3 300 rocprofv3 --kernel-trace --stats -d "$O/trace_c3" -o run --output-format csv \
  -- python3 "$R/bench.py" --config c3 --steps 20 --warmup 5 --no-cpu --no-verify --decode-inflight 1
CSV=$(find "$O/trace_c3" -name 'run_kernel_trace.csv' | head -1)
ALG=$(python3 -c "import json,sys; l=[json.loads(x) for x in open('$O/trace_c3.log') if x.startswith('{')][-1]; print(l['roofline']['algorithmic_bytes_per_launch'])")
step trace_c3_sum 60 python3 tools/trace_summary.py "$CSV" okv_tile_kernel 6 "$ALG" "$O/trace_c3.json" \
  "C3 one decode at a time (bench, 20 steps + 5 warmup + guard); two tile launches per decode" \
  --sha "$DSHA" --bench-log "$O/trace_c3.log" --per-step 2
cp "$O/trace_c3.json" profiles/r4/
step bench_c4 600 python3 bench.py --config c4
step bench_cz 600 python3 bench.py --config cz
step trace_cz 300 rocprofv3 --kernel-trace --stats -d "$O/trace_cz" -o run --output-format csv \
  -- python3 "$R/bench.py" --config cz --steps 10 --warmup 2 --no-cpu --no-verify --decode-inflight 1
step bench_c5 300 python3 bench.py --config c5 --no-cpu
step bench_c2 300 python3 bench.py --config c2 --no-cpu
step bench_cm 600 python3 bench.py --config cm
step bench_c1 300 python3 bench.py --config c1 --no-cpu
echo final done
