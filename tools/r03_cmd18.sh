set -o pipefail
mkdir -p gpurun_out
export FESOM2_LIB_NAME=libfesom2-accelerate.so
ROUNDS=2 STEPS=20 BENCH_ARGS="--no-check --kernel-timing all --config '127k x 47'" timeout -k 10 900 bash tools/sweep_env.sh "X=1 | --tracers 1" "X=1 | --tracers 2" "X=1 | --tracers 6" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_ntr_127k.txt
