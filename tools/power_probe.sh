#!/bin/bash
# Sample power and clocks while a long fused bench runs (is the march power-capped?).
# usage: tools/power_probe.sh <tag> [bench args...]   (env: VPTMCM_LIB, VPTMCM_MARCH_VARIANT)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
tag=$1; shift
timeout -k 10 120 python bench.py --steps 600000 --warmup 2048 --unfused-steps 0 --api-steps 0 \
  --general-steps 0 --cpu-seconds 0 "$@" > gpurun_out/pp_$tag.json 2> gpurun_out/pp_$tag.err &
pid=$!
sleep 5
for k in 1 2 3 4 5 6 7 8; do
  timeout -k 5 20 rocm-smi --showpower --showclocks >> gpurun_out/pp_$tag.smi 2>&1
  sleep 0.4
done
wait $pid
rc=$?
echo "$tag rc=$rc"
python3 - "$tag" <<'PY'
import re, sys
t = open(f"gpurun_out/pp_{sys.argv[1]}.smi").read()
w = [float(x) for x in re.findall(r"Package Power \(W\): ([0-9.]+)", t)]
c = [float(x) for x in re.findall(r"sclk clock level: \d+: \((\d+)Mhz\)", t)]
print(sys.argv[1], "power W", w, "sclk MHz", c)
PY
python3 -c "import json; d=json.load(open('gpurun_out/pp_$tag.json')); print('$tag', d['value'], d['roofline']['kernel_us_per_pass'])"
exit $rc
