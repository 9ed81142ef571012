R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/r3e
timeout -k 10 300 python3 bench.py --config c3 --no-cpu --no-verify > gpurun_out/r3e/bench_c3.log 2>&1 && tail -1 gpurun_out/r3e/bench_c3.log | cut -c1-300 &&
OKV_ABLATE=1 timeout -k 10 500 python3 tools/ablate_tile.py 8:16x 8:16xd1 8:16xd2 8:8x 8:16 > gpurun_out/r3e/ablate.log 2>&1; rc=$?; cat gpurun_out/r3e/ablate.log | grep -v amdgpu; [ $rc -ne 0 ] && exit $rc
OKV_ABLATE=1 timeout -k 10 300 python3 tools/zstd_prof.py 16384 > gpurun_out/r3e/zstd_prof.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/r3e/zstd_prof.log | tail -30; exit $rc
