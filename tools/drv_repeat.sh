#!/bin/bash
# The driver's round-end command line, repeated in fresh processes on one box:
# the spread of the credited line (value, kernel time, wall per step).
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/drv
: > gpurun_out/drv/lines.jsonl
for k in $(seq ${REPS:-5}); do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv/one.json 2>> gpurun_out/drv/err.txt || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/drv/one.json')); print(json.dumps({'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_avg_us': d['roofline']['kernel_avg_us'], 'region_wall_us': d['roofline']['region_wall_us'], 'wall_minus_kernel_us': d['roofline']['wall_minus_kernel_us'], 'frac': d['roofline']['frac']}))" >> gpurun_out/drv/lines.jsonl
done
cat gpurun_out/drv/lines.jsonl
