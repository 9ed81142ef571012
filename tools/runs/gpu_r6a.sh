#!/bin/bash
# Round 6: which stores give okv_tile_kernel its excess HBM writes on C3.
# The product tile pass with output classes left unwritten (ablation build,
# OKV_TILE=16xd<32+mask>, tile_pass kSkip): FETCH_SIZE / WRITE_SIZE and the
# EA request-size counters per arm, then the arms' times in one process.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r6a}; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -2 | cut -c1-300 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
for i in 1 2 3; do
  for L in r5 r6; do
    ABL_NBLK=256 ABL_KIND=0 ABL_BS=4096 ABL_TH=3584 ABL_ROUNDS=7 ABL_STEPS=50 \
      step ab_c2_${L}_$i 120 python3 tools/ab_lib.py tools/ab/r5/lib_dec$L.so $L
  done
done
step fused_phases 120 python3 tools/fused_phases.py
ARMS="8:16x 8:16xd32 8:16xd33 8:16xd34 8:16xd36 8:16xd40 8:16xd48 8:16xd63"
export ABL_ROUNDS=1 ABL_STEPS=2 ABL_CLASSES=1
for C in FETCH_SIZE WRITE_SIZE "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum"; do
  n=$(echo $C | cut -d' ' -f1)
  step pmc_$n 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/pmc_$n -o run -- python3 tools/ablate_tile.py $ARMS
done
step cal_w 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/cal_WRITE -o run -- tools/copybw3 cal
step cal_f 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/cal_FETCH -o run -- tools/copybw3 cal
export ABL_ROUNDS=5 ABL_STEPS=10
step time_arms 300 python3 tools/ablate_tile.py $ARMS
echo "r6a done"
