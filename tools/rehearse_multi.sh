#!/bin/bash
# Rehearse bench.py's N-rank path on a 1-GPU box: NPROC ranks (default 2) share cuda:0 over gloo
# (the driver's scaling run uses one rank per GPU over RCCL).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 ${REHEARSE_TIMEOUT:-600} python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NPROC:-2} --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus ${NPROC:-2} --steps 10 --warmup 3 --mapper-steps 3 --mapper-warmup 1 \
    --dist-backend gloo ${BENCH_ARGS:-} > gpurun_out/multi.json 2> gpurun_out/multi.err
rc=$?; echo "rc=$rc"; cat gpurun_out/multi.json; tail -5 gpurun_out/multi.err; exit $rc
