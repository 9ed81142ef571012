#!/bin/bash
# Copy the judged evidence of an end-of-round run (tools/runs/gpu_final6.sh) from
# gpurun_out/<tag>/ into profiles/r6/.
#   tools/runs/collect_r6.sh <tag>
set -e
cd "$(dirname "$0")/../.."
T=${1:-r6fin}
S=gpurun_out/$T
D=profiles/r6
mkdir -p $D
for f in $S/*.log; do
  [ -f "$f" ] && grep -v "amdgpu.ids" "$f" > $D/$(basename "$f")
done
for f in pmc_c3_full.json pmc_c4_encode.json trace_c3.json trace_cz.json trace_c5.json; do
  [ -f $S/$f ] && cp $S/$f $D/
done
for t in trace_c3 trace_cz trace_c4 trace_c5; do
  k=$(find $S/$t -name 'run_kernel_stats.csv' 2>/dev/null | head -1)
  [ -n "$k" ] && cp "$k" $D/${t}_kernel_stats.csv
done
for p in pmc_c3 pmc_c4; do
  for c in FETCH_SIZE WRITE_SIZE cal_FETCH cal_WRITE; do
    k=$(find $S/$p/$c -name 'run_counter_collection.csv' 2>/dev/null | head -1)
    [ -n "$k" ] && gzip -c "$k" > $D/${p}_${c}_counter_collection.csv.gz
  done
done
ls -la $D
