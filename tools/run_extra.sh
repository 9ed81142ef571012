#!/bin/bash
# Extra evidence: end-to-end pinned H2D -> decode -> D2H (C3), and kernel traces of CZ and C4.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O="$R/gpurun_out/extra"; mkdir -p "$O"
step() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > "$O/$n.log" 2>&1; local rc=$?; echo "[$n] exit $rc"; tail -2 "$O/$n.log" | cut -c1-400; [ $rc -ne 0 ] && exit $rc; return 0; }
step e2e 600 python3 bench.py --config c3 --e2e --no-cpu --no-verify --decode-inflight 1
step trace_cz 300 rocprofv3 --kernel-trace --stats -d "$O/trace_cz" -o run --output-format csv \
  -- python3 "$R/bench.py" --config cz --steps 10 --warmup 3 --no-cpu --no-verify --decode-inflight 1
step trace_c4 300 rocprofv3 --kernel-trace --stats -d "$O/trace_c4" -o run --output-format csv \
  -- python3 "$R/bench.py" --config c4 --steps 10 --warmup 3 --no-cpu --no-verify --c4-inflight 1
echo extra done
