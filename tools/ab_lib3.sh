#!/bin/bash
# Three-way alternating A/B of the default bench line: a library variant
# (VPTMCM_LIB=$LIB), the product with VPTMCM_SCHED_CACHE=0, and the product.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out; mkdir -p $OUT
for r in 1 2 3; do
  for arm in lib nocache prod; do
    case $arm in
      lib) env_="VPTMCM_LIB=${LIB:-pre}";;
      nocache) env_="VPTMCM_SCHED_CACHE=0";;
      prod) env_="VPTMCM_NONE=1";;
    esac
    env $env_ timeout -k 10 300 python bench.py --cpu-seconds 0 --js-steps 0 ${BENCH_ARGS:-} > $OUT/ab3_$arm.json 2>> $OUT/ab3.err || exit $?
    python3 -c "import json; d=json.load(open('$OUT/ab3_$arm.json')); r=d['roofline']; print(json.dumps({'arm': '$arm', 'value': d['value'], 'kern_us': r['kernel_avg_us'], 'unfused_us': d['unfused']['kernel_avg_us'], 'rgb_us': d['rgb']['kernel_us_per_pass'], 'general_us': d['general']['kernel_us_per_pass']}))" >> $OUT/ab3.jsonl
  done
done
cat $OUT/ab3.jsonl
