set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r03_gputests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r03_bench_default.json 2> gpurun_out/r03_bench_default.err || exit 1
timeout -k 10 300 python bench.py --tracers 6 --no-cpu-baseline > gpurun_out/r03_bench_6tr.json 2> gpurun_out/r03_bench_6tr.err || exit 1
timeout -k 10 300 python bench.py --config "127k x 47" --no-cpu-baseline > gpurun_out/r03_bench_127k.json 2> gpurun_out/r03_bench_127k.err || exit 1
