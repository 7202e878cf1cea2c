set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03d_smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03d_bench_default.json 2> gpurun_out/r03d_bench_default.err || exit 1
timeout -k 10 300 python bench.py --tracers 6 --no-cpu-baseline > gpurun_out/r03d_bench_6tr.json 2> gpurun_out/r03d_bench_6tr.err || exit 1
timeout -k 10 300 python bench.py --config "127k x 47" --no-cpu-baseline > gpurun_out/r03d_bench_127k.json 2> gpurun_out/r03d_bench_127k.err || exit 1
timeout -k 10 300 python bench.py --config "127k x 47" --tracers 6 --no-cpu-baseline > gpurun_out/r03d_bench_127k_6tr.json 2> gpurun_out/r03d_bench_127k_6tr.err || exit 1
timeout -k 10 300 python bench.py --path reference --no-cpu-baseline > gpurun_out/r03d_bench_reference_fast.json 2> gpurun_out/r03d_bench_reference_fast.err || exit 1
