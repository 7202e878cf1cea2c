set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r03_gputests_oddpad.log 2>&1 || exit 1
ROUNDS=3 STEPS=50 BENCH_ARGS="--no-check --kernel-timing all --config '127k x 47'" timeout -k 10 800 bash tools/sweep_env.sh "FESOM2_LIB_NAME=libfesom2-accelerate-old.so" "FESOM2_LIB_NAME=libfesom2-accelerate.so" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_oddpad_127k.txt
ROUNDS=2 STEPS=10 BENCH_ARGS="--no-check --kernel-timing all --config '127k x 47' --tracers 6" timeout -k 10 800 bash tools/sweep_env.sh "FESOM2_LIB_NAME=libfesom2-accelerate-old.so" "FESOM2_LIB_NAME=libfesom2-accelerate.so" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_oddpad_127k_6tr.txt
timeout -k 10 300 python bench.py --config "127k x 47" --no-cpu-baseline > gpurun_out/r03_oddpad_127k_check.json 2> gpurun_out/r03_oddpad_127k_check.err || exit 1
