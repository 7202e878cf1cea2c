set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --exchange host > gpurun_out/r03_n2_host.json 2> gpurun_out/r03_n2_host.err || exit 1
timeout -k 10 300 python bench.py --scaling strong --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03_strong_9p6m.json 2> gpurun_out/r03_strong_9p6m.err || exit 1
