cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for g in 256 768 1536; do OKV_ZSTD_EXEC_GRID=$g timeout -k 10 120 python -u tools/zstd_prof.py 4096 > gpurun_out/z3_$g.log 2>&1 || exit 1; echo "grid $g"; grep -E "exec|prof|stage" gpurun_out/z3_$g.log | tail -2; done
