#!/bin/bash
# Round-5 rocprofv3 evidence and the N > 1 rehearsal (one GPU box).  Each step bounded; the first
# failure ends the session.
#   1. kernel-trace stats + PMC read/write passes of the headline, 6 tracers and 9.6M x 80 on one GPU
#      (tools/profile.sh; profiles/pmc_traffic.py turns the PMC passes into traffic*.json)
#   2. the N > 1 bench path with 2 ranks on this one GPU (host halo: RCCL refuses two ranks on one
#      device), headline + strong leg, every rank checking its outputs
set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 900 bash tools/profile.sh r05_1p2M
echo "profile 1.2M done"
BENCH_ARGS="--tracers 6" timeout -k 10 900 bash tools/profile.sh r05_6tr
echo "profile 6tr done"
BENCH_ARGS="--scaling strong" timeout -k 10 1000 bash tools/profile.sh r05_9p6M
echo "profile 9.6M done"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29531 bench.py --gpus 2 --exchange host --extras on --steps 10 --warmup 2 \
    > gpurun_out/r05_bench_n2_hostexchange_rehearsal.json 2> gpurun_out/r05_bench_n2_hostexchange_rehearsal.err
echo "n2 rehearsal done"
