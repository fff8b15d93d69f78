#!/bin/bash
# Deal-reuse A/B: the GPU tests that cover it (SKIP_TESTS=1: none), then the
# driver's command alternating VPTMCM_SCHED_CACHE=1 / 0, one JSON line per run.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out; mkdir -p $OUT
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_knobs.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_group.py > $OUT/sched_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -2 $OUT/sched_tests.log
  [ $rc -ne 0 ] && exit $rc
fi
for v in 1 0 1 0 1 0; do
  VPTMCM_SCHED_CACHE=$v timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --js-steps 0 > $OUT/ab_$v.json 2>> $OUT/ab.err || exit $?
  python3 -c "import json; d=json.load(open('$OUT/ab_$v.json')); r=d['roofline']; u=d['unfused']; print(json.dumps({'cache': $v, 'value': d['value'], 'kern_us': r['kernel_avg_us'], 'wmk': r['wall_minus_kernel_us'], 'unfused_kern_us': u['kernel_avg_us'], 'unfused_value': u['value']}))" >> $OUT/ab_sched.jsonl
done
cat $OUT/ab_sched.jsonl
