#!/bin/bash
# round 6 session 12: the N > 1 bench path rehearsed on one GPU with the host halo (RCCL refuses two
# ranks on one device): 2 ranks on the default workload (large partitions), 4 ranks at 127k x 47
# per rank (union plans with halo columns in the unions) plus the strong leg split over 4
set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29531 bench.py --gpus 2 --exchange host --extras on --steps 10 --warmup 2 \
    > gpurun_out/s12_bench_n2_hostexchange.json 2> gpurun_out/s12_bench_n2_hostexchange.err
echo "n2 done"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 4 --exchange host --extras on --config '127k x 47' --strong-config '1.2M x 80' \
    --steps 20 --warmup 3 > gpurun_out/s12_bench_n4_hostexchange_127k.json 2> gpurun_out/s12_bench_n4_hostexchange_127k.err
echo "n4 done"
