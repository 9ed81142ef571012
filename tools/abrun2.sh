cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab2_test.log 2>&1; rc=$?; tail -3 gpurun_out/ab2_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c2 --no-cpu > gpurun_out/ab2_c2.log 2>&1 || exit 1; tail -1 gpurun_out/ab2_c2.log | grep -o '"value[^,]*\|"ms_per_step[^,]*\|"kernel_ms[^}]*'
timeout -k 10 300 python -u bench.py --config c3 --no-cpu > gpurun_out/ab2_c3.log 2>&1 || exit 1; tail -1 gpurun_out/ab2_c3.log | grep -o '"value[^,]*\|"kernel_ms[^}]*'
timeout -k 10 300 python -u bench.py --config cm --steps 5 --warmup 2 > gpurun_out/ab2_cm.log 2>&1 || exit 1; tail -1 gpurun_out/ab2_cm.log | grep -o '"value[^,]*\|"stage_ms[^}]*'
