#!/bin/bash
# PMC passes behind bench.py's roofline fields (one rocprofv3 pass per counter
# group, --kernel-trace only beside --pmc, each under its own time limit):
#   req   TCC read requests by size (32/64/128 B) -> memory-side read bytes
#   fetch FETCH_SIZE + DRAM-bound read requests
#   write WRITE_SIZE
#   sq    VALU/SALU issue + wave cycles + GRBM clock
# for the known-bytes gather (tools/gather_calib) and for bench.py's timed
# launch at the pass counts in PPL (default: the driver's 20 and the default 32).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${PMC_OUT:-gpurun_out/pmcreq}
mkdir -p $OUT
declare -A G=(
  [req]="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
  [fetch]="FETCH_SIZE TCC_EA0_RDREQ_DRAM_sum"
  [write]="WRITE_SIZE"
  [sq]="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE"
)
run() {  # name, group, cmd...
  local name=$1 grp=$2
  shift 2
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc ${G[$grp]} \
      -d "$GRAFT_REPO_ROOT/$OUT/${name}_$grp" -o run --output-format csv -- "$@" \
      > "$GRAFT_REPO_ROOT/$OUT/${name}_$grp.out" 2> "$GRAFT_REPO_ROOT/$OUT/${name}_$grp.err")
  local rc=$?
  echo "$name $grp rc=$rc" | tee -a $OUT/status.txt
  [ $rc -le 5 ]
}
for grp in ${CALIB_GROUPS-req fetch}; do
  run calib "$grp" "$GRAFT_REPO_ROOT/tools/gather_calib" 1024 || exit 1
done
for ppl in ${PPL:-20 32}; do
  for grp in ${GROUPS_BENCH:-req fetch write sq}; do
    run "bench$ppl" "$grp" python3 "$GRAFT_REPO_ROOT/bench.py" --steps $ppl --warmup 64 --unfused-steps 0 \
        --api-steps 0 --general-steps 0 --rgb-steps 0 --js-steps 0 --settle-ms 0 --cpu-seconds 0 ${BENCH_ARGS:-} || exit 1
  done
done
exit 0
