cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/snap_test.log 2>&1; rc=$?; tail -25 gpurun_out/snap_test.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/snap_smoke.log 2>&1 || exit $?
tail -3 gpurun_out/snap_smoke.log; exit $rc
