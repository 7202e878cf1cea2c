set -o pipefail
mkdir -p gpurun_out
export FESOM2_LIB_NAME=libfesom2-accelerate.so
ROUNDS=3 STEPS=50 BENCH_ARGS="--no-check --kernel-timing all --config '127k x 47'" timeout -k 10 800 bash tools/sweep_env.sh "X=1" "FESOM2_P1V_B3H=1" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_oddpad_int_127k.txt
ROUNDS=2 STEPS=10 BENCH_ARGS="--no-check --kernel-timing all --config '127k x 47' --tracers 6" timeout -k 10 800 bash tools/sweep_env.sh "X=1" "FESOM2_P1V_B3H=1" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_oddpad_int_127k_6tr.txt
