#!/bin/bash
# Diagnostic counter passes (run on the GPU box via gpurun): SQ wave-state
# cycles, L2 miss traffic and its average queue level (latency by Little's
# law), TA stalls -- each group in its own rocprofv3 run (slot limits).
#   tools/pmc_diag.sh <tag> <program> [args...]     (program: python3 or a binary)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
TAG=$1
shift
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM" \
         "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_HIT_sum TCC_MISS_sum" \
         "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_128B_sum" \
         "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM"; do
  i=$((i + 1))
  timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/p$i" -o run \
    -- "$@" > "$OUT/p$i.log" 2>&1
  rc=$?; echo "[pass $i] exit $rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
