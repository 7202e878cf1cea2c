set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py -m gpu -x -q --timeout 200 --timeout-method thread -k "reference or fast_mode or full_pass or graph or half_pass or thread" > gpurun_out/r03_fast.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --path reference --no-cpu-baseline > gpurun_out/r03_ref_fast.json 2> gpurun_out/r03_ref_fast.err || exit 1
for p in 16384 4096 2048 1024; do
  FESOM2_PATCH=$p timeout -k 10 200 python bench.py --tracers 6 --no-cpu-baseline --no-check --steps 10 > gpurun_out/r03_6tr_p$p.json 2> gpurun_out/r03_6tr_p$p.err || exit 1
done
