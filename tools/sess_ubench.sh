#!/bin/bash
# Instruction-cost micro-benchmark + instruction-count PMC for two camera poses.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 120 tools/ubench > gpurun_out/ubench.txt 2>&1 || exit $?
printf 'SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM\nSQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU\nSQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAVES\n' > /tmp/groups.txt
BENCH_ARGS="--camera near" bash tools/pmc.sh /tmp/groups.txt > gpurun_out/pmc_near.log 2>&1 || exit $?
mv gpurun_out/pmc gpurun_out/pmc_near
BENCH_ARGS="--camera default" bash tools/pmc.sh /tmp/groups.txt > gpurun_out/pmc_default.log 2>&1 || exit $?
mv gpurun_out/pmc gpurun_out/pmc_default
