#!/bin/bash
# SQ instruction counters of the march for several bench configurations
# (one rocprofv3 --pmc pass each); usage: pmc_cfgs.sh "<args1>" "<args2>" ...
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/pmc_cfgs
i=0
for args in "$@"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_cfgs/c$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 2 --cpu-seconds 0 $args > "$GRAFT_REPO_ROOT/gpurun_out/pmc_cfgs/c$i.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/pmc_cfgs/c$i.err")
  rc=$?; echo "cfg $i ($args) rc=$rc"
  [ $rc -gt 5 ] && exit $rc
done
exit 0
