#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out; mkdir -p $OUT
for v in 1 0 1 0; do
  VPTMCM_SCHED_CACHE=$v timeout -k 10 300 python bench.py --cpu-seconds 0 --js-steps 0 > $OUT/abd_$v.json 2>> $OUT/abd.err || exit $?
  python3 -c "import json; d=json.load(open('$OUT/abd_$v.json')); r=d['roofline']; print(json.dumps({'cache': $v, 'value': d['value'], 'kern_us': r['kernel_avg_us'], 'wmk': r['wall_minus_kernel_us'], 'rgb_us_per_pass': d['rgb']['kernel_us_per_pass'], 'general_us_per_pass': d['general']['kernel_us_per_pass']}))" >> $OUT/ab_default.jsonl
done
cat $OUT/ab_default.jsonl
