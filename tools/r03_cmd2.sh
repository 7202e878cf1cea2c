set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "reference or fast_mode or full_pass" > gpurun_out/r03_fast2.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --path reference --no-cpu-baseline > gpurun_out/r03_ref_fast2.json 2> gpurun_out/r03_ref_fast2.err || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r03_split2.json 2> gpurun_out/r03_split2.err || exit 1
timeout -k 10 100 ./tools/stream_probe 126976 47 > gpurun_out/r03_stream127k.txt 2>&1 || exit 1
