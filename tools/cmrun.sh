cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --config cm --steps 5 --warmup 2 > gpurun_out/cm_bench.log 2>&1 || { tail -30 gpurun_out/cm_bench.log; exit 1; }
tail -2 gpurun_out/cm_bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/cm_prof -o cm --output-format csv -- python3 bench.py --config cm --steps 3 --warmup 1 > gpurun_out/cm_prof.log 2>&1; rc=$?
f=$(find gpurun_out/cm_prof -name 'cm_kernel_stats.csv' | head -1); cut -d, -f1-4 $f | head -30
exit $rc
