set -o pipefail
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
ROUNDS=3 STEPS=30 BENCH_ARGS="--no-check" timeout -k 10 900 bash tools/sweep_env.sh "FESOM2_ALLOC_SKEW=0" "FESOM2_ALLOC_SKEW=4352" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_skew_1p2m.txt
ROUNDS=2 STEPS=30 BENCH_ARGS="--no-check --config '127k x 47'" timeout -k 10 600 bash tools/sweep_env.sh "FESOM2_ALLOC_SKEW=0" "FESOM2_ALLOC_SKEW=4352" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_skew_127k.txt
ROUNDS=1 STEPS=10 BENCH_ARGS="--no-check --tracers 6" timeout -k 10 600 bash tools/sweep_env.sh "FESOM2_ALLOC_SKEW=0" "FESOM2_ALLOC_SKEW=4352" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_skew_6tr.txt
