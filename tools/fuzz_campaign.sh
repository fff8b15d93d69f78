#!/bin/bash
# A long randomised parity campaign on the GPU box: the random-configuration
# tests of tests/test_gpu_fuzz.py over fresh draws (VPTMCM_FUZZ_BASE) and many
# more of them (VPTMCM_FUZZ_CASES spectral cases, half as many RGB cases, a
# quarter as many Mode B band cases, an eighth as many device-list composites,
# and CASES/16 random operation sequences, tests/test_gpu_sequences.py, unless
# SEQ says), every one bit for bit against the oracle.
#   CASES=1200 BASE=100000 bash tools/fuzz_campaign.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
C=${CASES:-1200}
VPTMCM_FUZZ_CASES=$C VPTMCM_FUZZ_BASE=${BASE:-100000} \
VPTMCM_SEQ_CASES=${SEQ:-$((C / 16))} VPTMCM_SEQ_BASE=${BASE:-100000} \
  timeout -k 10 ${FUZZ_T:-1000} python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_sequences.py -m gpu -v --maxfail=5 \
  --timeout 120 --timeout-method thread -k "random" -p no:cacheprovider > $OUT/fuzz_campaign.log 2>&1
rc=$?
echo "fuzz rc=$rc" | tee -a $OUT/status.txt
tail -3 $OUT/fuzz_campaign.log
exit $rc
