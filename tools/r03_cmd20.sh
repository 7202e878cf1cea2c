set -o pipefail
mkdir -p gpurun_out
ROUNDS=2 STEPS=20 BENCH_ARGS="--no-check --kernel-timing all" timeout -k 10 600 bash tools/sweep_env.sh "X=1" "FESOM2_P1V_BATCH=23" "FESOM2_P1V_BATCH=32" "FESOM2_P1V_BATCH=33" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_p1vbatch_1tr.txt
ROUNDS=1 STEPS=10 BENCH_ARGS="--no-check --kernel-timing all --tracers 6" timeout -k 10 600 bash tools/sweep_env.sh "X=1" "FESOM2_P1V_BATCH=23" "FESOM2_P1V_BATCH=33" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_p1vbatch_6tr.txt
FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so FESOM2_P1V_BATCH=33 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/r03_p1vb33_check.json 2> gpurun_out/r03_p1vb33_check.err || exit 1
