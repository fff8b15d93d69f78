#!/bin/bash
# Round-end evidence on one box: GPU tests, the default bench line, a rocprofv3
# kernel-trace summary of the same command, and FETCH_SIZE / WRITE_SIZE passes
# (one counter per pass) for the bench workload and for a calibration launch
# whose bytes are known (S = 0, one pass per launch: photon state in + out,
# image + flags out, no volume gathers).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
fault() { case $1 in 0|1|2|3|4|5) return 1;; *) return 0;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; fault $rc && exit $rc
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; fault $rc && exit $rc
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --cpu-seconds 0 > "$GRAFT_REPO_ROOT/$OUT/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof.err")
rc=$?; echo "prof rc=$rc"; fault $rc && exit $rc
for cfg in "bench|--steps 32 --warmup 32 --unfused-steps 0 --api-steps 0 --cpu-seconds 0" "calib|--steps 32 --warmup 16 --unfused-steps 0 --api-steps 0 --cpu-seconds 0 --fuse 1 --photon-steps 0"; do
  name=${cfg%%|*}; args=${cfg#*|}
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d "$GRAFT_REPO_ROOT/$OUT/pmc_${name}_$c" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" $args > "$GRAFT_REPO_ROOT/$OUT/pmc_${name}_$c.json" 2> "$GRAFT_REPO_ROOT/$OUT/pmc_${name}_$c.err")
    rc=$?; echo "pmc $name $c rc=$rc"; fault $rc && exit $rc
  done
done
exit 0
