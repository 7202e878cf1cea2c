set -o pipefail
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
ROUNDS=2 STEPS=30 BENCH_ARGS="--no-check" timeout -k 10 600 bash tools/sweep_env.sh "FESOM2_P1V_WAVES=0" "FESOM2_P1V_WAVES=8" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_waves_1p2m.txt
ROUNDS=2 STEPS=50 BENCH_ARGS="--no-check --config '127k x 47'" timeout -k 10 600 bash tools/sweep_env.sh "FESOM2_P1V_WAVES=0" "FESOM2_P1V_WAVES=7" "FESOM2_P1V_WAVES=8" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_waves_127k.txt
FESOM2_P1V_WAVES=8 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/r03_w8_check.json 2>gpurun_out/r03_w8_check.err || exit 1
FESOM2_P1V_WAVES=8 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --config "127k x 47" > gpurun_out/r03_w8_127k_check.json 2>gpurun_out/r03_w8_127k_check.err || exit 1
unset FESOM2_LIB_NAME
timeout -k 10 100 ./tools/stream_probe 126976 47 > gpurun_out/r03_stream127k_b.txt 2>&1 || exit 1
timeout -k 10 100 ./tools/stream_probe 126976 48 >> gpurun_out/r03_stream127k_b.txt 2>&1 || exit 1
timeout -k 10 100 ./tools/stream_probe 1200000 80 >> gpurun_out/r03_stream127k_b.txt 2>&1 || exit 1
