#!/bin/bash
# Rehearse the N > 1 bench path on a one-GPU box: two ranks pinned to device 0
# (RCCL may refuse duplicate devices; the log says which step failed).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export VPTMCM_BENCH_DEVICE=0 NCCL_DEBUG=WARN
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 2 --steps 32 --warmup 16 --cpu-seconds 0 > gpurun_out/mr2.json 2> gpurun_out/mr2.err
echo "rc=$?"; cat gpurun_out/mr2.json; tail -30 gpurun_out/mr2.err
