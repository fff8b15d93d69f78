#!/bin/bash
# The driver's command line, alternating the region's begin event: stamped by
# the first launch's dispatch (default) vs a marker recorded just before it.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/tb
: > gpurun_out/tb/lines.jsonl
for k in $(seq ${REPS:-4}); do
  for mode in stamp marker; do
    VPTMCM_TIME_BEGIN=$mode timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --js-steps 0 > gpurun_out/tb/one.json 2>> gpurun_out/tb/err.txt || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/tb/one.json')); print(json.dumps({'begin': sys.argv[1], 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_avg_us': d['roofline']['kernel_avg_us']}))" $mode >> gpurun_out/tb/lines.jsonl
  done
done
cat gpurun_out/tb/lines.jsonl
