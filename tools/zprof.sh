cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
N=${1:-16384}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/zp -o zp --output-format csv -- python3 tools/zstd_prof.py $N > gpurun_out/zp.log 2>&1; rc=$?
tail -4 gpurun_out/zp.log
f=$(find gpurun_out/zp -name 'zp_kernel_stats.csv' | head -1); cut -d, -f1-8 $f | head -20
exit $rc
