set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batched.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread -k "reference or fast_mode or full_pass or batched or config3" > gpurun_out/r03_t3.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --path reference --no-cpu-baseline > gpurun_out/r03_ref_fast2.json 2> gpurun_out/r03_ref_fast2.err || exit 1
timeout -k 10 100 ./tools/stream_probe 126976 47 > gpurun_out/r03_stream127k.txt 2>&1 || exit 1
for r in 1 2; do
timeout -k 10 200 python bench.py --tracers 6 --no-cpu-baseline --no-check --steps 10 > gpurun_out/r03_6tr_tl_$r.json 2> gpurun_out/r03_6tr_tl_$r.err || exit 1
FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so FESOM2_P1V_TLOOP=0 timeout -k 10 200 python bench.py --tracers 6 --no-cpu-baseline --no-check --steps 10 > gpurun_out/r03_6tr_notl_$r.json 2> gpurun_out/r03_6tr_notl_$r.err || exit 1
done
