set -o pipefail
mkdir -p gpurun_out
ROUNDS=2 STEPS=10 BENCH_ARGS="--no-check --kernel-timing all --tracers 6" timeout -k 10 800 bash tools/sweep_env.sh "X=1" "FESOM2_PATCH=1024" "FESOM2_PATCH=1024 FESOM2_ABLATE=1" "FESOM2_PATCH=512" "FESOM2_PATCH=256" "FESOM2_PATCH=2048" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_patch_6tr.txt
ROUNDS=2 STEPS=20 BENCH_ARGS="--no-check --kernel-timing all" timeout -k 10 500 bash tools/sweep_env.sh "X=1" "FESOM2_PATCH=1024" "FESOM2_PATCH=512" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_patch_1tr.txt
