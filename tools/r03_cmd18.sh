set -o pipefail
mkdir -p gpurun_out
export FESOM2_LIB_NAME=libfesom2-accelerate.so
ROUNDS=2 STEPS=10 BENCH_ARGS="--no-check --kernel-timing all" timeout -k 10 900 bash tools/sweep_env.sh "X=1 | --tracers 1" "X=1 | --tracers 2" "X=1 | --tracers 3" "X=1 | --tracers 6" "X=1 | --tracers 2 --config '127k x 47'" "X=1 | --tracers 6 --config '127k x 47'" "X=1 | --tracers 1 --config '127k x 47'" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_ntr.txt
