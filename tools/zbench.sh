cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/zb_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/zb_pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --config cz > gpurun_out/zb_bench_cz.log 2>&1 || exit $?; tail -1 gpurun_out/zb_bench_cz.log
