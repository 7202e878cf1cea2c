set -o pipefail
mkdir -p gpurun_out
ROUNDS=2 STEPS=10 BENCH_ARGS="--no-check --kernel-timing all --tracers 6" timeout -k 10 900 bash tools/sweep_env.sh "X=1" "FESOM2_GROUP_SHIFT=-1" "FESOM2_GROUP_SHIFT=-1 FESOM2_P1V_B3H=0" "FESOM2_GROUP_SHIFT=-2" "FESOM2_GROUP_SHIFT=-1 FESOM2_PATCH=1024" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_group2_6tr.txt
ROUNDS=2 STEPS=10 BENCH_ARGS="--no-check --kernel-timing all --tracers 2" timeout -k 10 600 bash tools/sweep_env.sh "X=1" "FESOM2_GROUP_SHIFT=-1" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_group_2tr.txt
ROUNDS=2 STEPS=20 BENCH_ARGS="--no-check --kernel-timing all" timeout -k 10 600 bash tools/sweep_env.sh "X=1" "FESOM2_GROUP_SHIFT=-1" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_group_1tr.txt
