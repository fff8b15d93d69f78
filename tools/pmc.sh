#!/bin/bash
# Collect PMC counter groups for the march kernel (one rocprofv3 pass per group,
# --kernel-trace only beside --pmc, as the pool requires).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/pmc
[ -n "${LIST:-}" ] && (rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true)
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc $group -d "$GRAFT_REPO_ROOT/gpurun_out/pmc/g$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 32 --warmup 16 --unfused-steps 0 --cpu-seconds 0 ${BENCH_ARGS:-} > "$GRAFT_REPO_ROOT/gpurun_out/pmc/g$i.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/pmc/g$i.err")
  rc=$?; echo "group $i ($group) rc=$rc"
  [ $rc -gt 5 ] && exit $rc
done < "${1:-tools/pmc_groups.txt}"
exit 0
