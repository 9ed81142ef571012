#!/bin/bash
# CM decode stage: small-block decodes in pieces (ablation build, OKV_SMALL_PIECE_MB)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-cmpiece}; mkdir -p $O
OKV_ABLATE=1 OKV_SMALL_PIECE_MB=1 timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py -m gpu -q \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "[tests, 1 MiB pieces] exit $rc: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for mb in 0 48 96 192 384; do
  OKV_ABLATE=1 OKV_SMALL_PIECE_MB=$mb timeout -k 10 300 python3 bench.py --config cm --no-cpu --steps 10 --warmup 2 > $O/mb_${mb}_$r.log 2>&1
  rc=$?; echo "[piece $mb MiB run $r] exit $rc $(grep -o '"stage_ms": {[^}]*}\|"frac": [0-9.]*\|"value": [0-9.]*' $O/mb_${mb}_$r.log | tr '\n' ' ')"; [ $rc -ne 0 ] && exit $rc
done
done
exit 0
