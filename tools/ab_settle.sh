#!/bin/bash
# The driver's command line, alternating the clock-settling time before the
# timed region (--settle-ms): the credited line's level and spread.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/st2
: > gpurun_out/st2/lines.jsonl
for k in $(seq ${REPS:-4}); do
  for ms in ${SETTLES:-150 400}; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --js-steps 0 --settle-ms $ms > gpurun_out/st2/one.json 2>> gpurun_out/st2/err.txt || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/st2/one.json')); print(json.dumps({'settle_ms': int(sys.argv[1]), 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_avg_us': d['roofline']['kernel_avg_us']}))" $ms >> gpurun_out/st2/lines.jsonl
  done
done
cat gpurun_out/st2/lines.jsonl
