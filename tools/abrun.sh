cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_test.log 2>&1; rc=$?; tail -3 gpurun_out/ab_test.log; [ $rc -eq 0 ] || exit $rc
for nt in 64 256; do
  OKV_GATHER_THREADS=$nt timeout -k 10 300 python -u bench.py --config cm --steps 5 --warmup 2 > gpurun_out/ab_cm_$nt.log 2>&1 || exit 1
  echo "cm nt=$nt"; tail -1 gpurun_out/ab_cm_$nt.log | cut -c1-200; tail -1 gpurun_out/ab_cm_$nt.log | grep -o '"stage_ms.*'
done
timeout -k 10 300 python -u bench.py --config c2 --no-cpu > gpurun_out/ab_c2.log 2>&1 || exit 1; tail -1 gpurun_out/ab_c2.log | grep -o '"ms_per_step[^,]*\|"kernel_ms[^}]*'
timeout -k 10 300 python -u bench.py --config c3 --no-cpu > gpurun_out/ab_c3.log 2>&1 || exit 1; tail -1 gpurun_out/ab_c3.log | grep -o '"value[^,]*\|"kernel_ms[^}]*'
