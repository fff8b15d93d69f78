#!/bin/bash
# GPU session: parity tests first (stop on a fault-class exit), then a sweep file.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -gt 5 ] && exit $rc
bash tools/sweep.sh "${1:-tools/sweep.txt}"
