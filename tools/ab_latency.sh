#!/bin/bash
# A/B of one-launch regions (tools/launch_latency.py, medians of 40 regions)
# between library variants on one box: LIBS="base product" (product = the
# in-tree libvptmcm.so), PASSES="20 1", REPS rounds, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/ab
: > gpurun_out/ab/lat.jsonl
for rep in $(seq ${REPS:-4}); do
  for lib in ${LIBS:-base product}; do
    for F in ${PASSES:-20 1}; do
      if [ $lib = product ]; then e="VPTMCM_X=0"; else e="VPTMCM_LIB=$lib"; fi
      out=$(timeout -k 10 120 env $e python3 tools/launch_latency.py --passes $F --regions 40 2>>gpurun_out/ab/err.txt) || exit 1
      echo "{\"lib\": \"$lib\", \"F\": $F, \"r\": $out}" >> gpurun_out/ab/lat.jsonl
    done
  done
done
