#!/bin/bash
# tools/brick_gather: sample rates per table size and mode, then the L2's fabric
# read requests for the two candidate footprints.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/brick
mkdir -p $OUT
: > $OUT/rates.jsonl
for c in "0 512" "1 182" "0 182" "0 64" "1 64" "0 1024" "1 512" "0 512" "1 182"; do
  timeout -k 10 60 tools/brick_gather $c >> $OUT/rates.jsonl || exit 1
done
for c in "0 512" "1 182"; do
  set -- $c
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
      -d "$GRAFT_REPO_ROOT/$OUT/req_$1_$2" -o run --output-format csv -- "$GRAFT_REPO_ROOT/tools/brick_gather" $1 $2 \
      > /dev/null 2> "$GRAFT_REPO_ROOT/$OUT/req_$1_$2.err") || exit 1
done
cat $OUT/rates.jsonl
