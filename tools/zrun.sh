cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_zstd_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/z_test.log 2>&1; rc=$?; tail -15 gpurun_out/z_test.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/zstd_prof.py 4096 > gpurun_out/z_prof.log 2>&1; rc=$?; tail -5 gpurun_out/z_prof.log; exit $rc
