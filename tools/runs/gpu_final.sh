#!/bin/bash
# End-of-round evidence at the committed sources (run on the GPU box via gpurun):
#   1. GPU suite + smoke
#   2. C3 PMC passes (FETCH_SIZE / WRITE_SIZE + 4 GiB calibration), summarised with the decode
#      sources' SHA into profiles/r3/pmc_c3_full.json (so the bench below attaches traffic)
#   3. C4 PMC passes -> profiles/r3/pmc_c4_encode.json (encode sources' SHA)
#   4. the driver's bench command (C3, CPU baseline included), then the C3 kernel trace one
#      decode at a time
#   5. the other configurations' bench lines
# Every step has its own time limit; the first failure ends the script.
#   tools/gpu_final.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
T=${1:-final}
O="$R/gpurun_out/$T"
mkdir -p "$O"
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
step pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
DSHA=$(python3 -c "import bench; print(bench.source_sha(bench.DECODE_SOURCES))")
ESHA=$(python3 -c "import bench; print(bench.source_sha(bench.ENCODE_SOURCES))")
step pmc_c3 600 "$R/tools/pmc_run.sh" "$T/pmc_c3" bench.py --config c3 --steps 3 --warmup 1 \
  --no-cpu --no-verify --decode-inflight 1
step pmc_c3_sum 60 python3 tools/pmc_summary.py "$O/pmc_c3" "$O/pmc_c3_full.json" \
  "{\"source_sha\": \"$DSHA\", \"config\": \"c3\", \"mode\": \"full\", \"source\": \"gpurun_out/$T/pmc_c3\"}"
step pmc_c4 600 "$R/tools/pmc_run.sh" "$T/pmc_c4" bench.py --config c4 --steps 3 --warmup 1 \
  --no-cpu --no-verify --c4-inflight 1
step pmc_c4_sum 60 python3 tools/pmc_summary.py "$O/pmc_c4" "$O/pmc_c4_encode.json" \
  "{\"source_sha\": \"$ESHA\", \"config\": \"c4\", \"mode\": \"encode\", \"source\": \"gpurun_out/$T/pmc_c4\"}"
cp "$O/pmc_c3_full.json" "$O/pmc_c4_encode.json" profiles/r3/
step bench_driver 600 python3 bench.py --gpus 1 --steps 20 --warmup 5
step trace_c3 300 rocprofv3 --kernel-trace --stats -d "$O/trace_c3" -o run --output-format csv \
  -- python3 "$R/bench.py" --config c3 --steps 20 --warmup 5 --no-cpu --no-verify --decode-inflight 1
step bench_c4 600 python3 bench.py --config c4
step bench_cz 600 python3 bench.py --config cz
step bench_c5 300 python3 bench.py --config c5 --no-cpu
step bench_c2 300 python3 bench.py --config c2 --no-cpu
step bench_cm 600 python3 bench.py --config cm
step bench_c1 300 python3 bench.py --config c1 --no-cpu
echo final done
