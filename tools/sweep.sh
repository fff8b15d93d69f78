#!/bin/bash
# Diagnostic sweep: one bench line per configuration (kernel time vs S, TF, layout).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
: > gpurun_out/sweep.jsonl
: > gpurun_out/sweep_full.jsonl
while read -r args; do
  [ -z "$args" ] && continue
  envs=""; rest="$args"
  if [[ "$args" == *";"* ]]; then envs="${args%%;*}"; rest="${args#*;}"; fi
  timeout -k 10 300 env $envs python bench.py --steps 512 --warmup 2048 --unfused-steps 0 --api-steps 0 --general-steps 0 --rgb-steps 0 --js-steps 0 --cpu-seconds 0 $rest > gpurun_out/one.json 2>> gpurun_out/sweep.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "{\"args\": \"$args\", \"rc\": $rc}" >> gpurun_out/sweep.jsonl; [ $rc -gt 5 ] && exit $rc; continue; fi
  python3 -c "import json,sys; print(json.dumps({'args': sys.argv[1], 'line': json.load(open('gpurun_out/one.json'))}))" "$args" >> gpurun_out/sweep_full.jsonl
  python3 -c "import json,sys; d=json.load(open('gpurun_out/one.json')); print(json.dumps({'args': sys.argv[1], 'value': d['value'], 'kern_us': d['roofline']['kernel_avg_us'], 'us_pass': d['roofline'].get('kernel_us_per_pass'), 'ms_step': d['ms_per_step'], 'frac': d['roofline']['frac']}))" "$args" >> gpurun_out/sweep.jsonl
done < "${1:-tools/sweep.txt}"
cat gpurun_out/sweep.jsonl
