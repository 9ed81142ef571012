cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for n in 256 1024 2048; do timeout -k 10 120 python -u tools/zstd_prof.py $n > gpurun_out/z_prof_$n.log 2>&1 || exit 1; tail -2 gpurun_out/z_prof_$n.log; done
