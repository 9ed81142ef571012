#!/bin/bash
# Round 6: zstd sequence-stage counters, product build vs the cached-load
# timing bound (lib_zstfix): SQ wave states, L2, TA and TCP (vector L1 / its
# TLB) passes, one rocprofv3 run per group (slot limits), CZ one decode at a time.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r6r}; mkdir -p $O
timeout -k 5 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
TCP=""
for c in TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_PENDING_STALL_CYCLES_sum; do
  grep -q "\b${c%_sum}\b" $O/avail.txt && TCP="$TCP $c"
done
echo "TCP counters: $TCP"
for L in product zstfix; do
  LIBENV=""; [ $L = zstfix ] && LIBENV=tools/ab/r5/lib_zstfix.so; mkdir -p $O/$L
  i=0
  for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum" \
           "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU" \
           "$TCP"; do
    i=$((i + 1))
    [ -z "${C// /}" ] && continue
    OKV_LIB=$LIBENV timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$O/$L/p$i" -o run \
      -- python3 bench.py --config cz --steps 2 --warmup 1 --no-cpu --no-verify --decode-inflight 1 > "$O/$L/p$i.log" 2>&1
    rc=$?; echo "[$L pass $i] exit $rc"; [ $rc -ne 0 ] && [ $L = product ] && exit $rc
  done
  python3 tools/pmc_diag_summary.py $O/$L zstd_seq > $O/$L/summary.txt 2>&1
done
echo "r6r done"
