#!/bin/bash
# Scattered 8-B gathers (tools/gather_calib, 1 GiB table) with each load
# cache-policy flavour: rate, then the L2's fabric read requests by size.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/gflav
mkdir -p $OUT
: > $OUT/rates.jsonl
for v in 0 1 2 3 4; do
  timeout -k 10 60 tools/gather_calib 1024 256 4096 $v >> $OUT/rates.jsonl || exit 1
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
      -d "$GRAFT_REPO_ROOT/$OUT/req_$v" -o run --output-format csv -- "$GRAFT_REPO_ROOT/tools/gather_calib" 1024 256 4096 $v \
      > /dev/null 2> "$GRAFT_REPO_ROOT/$OUT/req_$v.err") || exit 1
done
cat $OUT/rates.jsonl
