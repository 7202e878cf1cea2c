set -o pipefail
mkdir -p gpurun_out
ROUNDS=2 STEPS=10 BENCH_ARGS="--no-check --kernel-timing all --tracers 6" timeout -k 10 900 bash tools/sweep_env.sh "X=1" "FESOM2_GROUP_SHIFT=-1" "FESOM2_GROUP_SHIFT=1" "FESOM2_PATCH=1024 FESOM2_GROUP_SHIFT=1" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_group_6tr.txt
