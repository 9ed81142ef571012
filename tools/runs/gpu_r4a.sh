#!/bin/bash
# round-4 parity check: selected GPU test files (default: decode / zstd / reader / encode)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
TAG=${1:-r4a}
shift
FILES=${*:-tests/test_encode_gpu.py tests/test_zstd_gpu.py tests/test_decode_gpu.py tests/test_reader_gpu.py}
timeout -k 10 1000 python -u -m pytest $FILES -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
echo "pytest exit $rc"
grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_pytest.log | tail -40
exit $rc
