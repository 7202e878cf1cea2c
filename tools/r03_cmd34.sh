set -o pipefail
mkdir -p gpurun_out
ROUNDS=3 STEPS=50 BENCH_ARGS="--no-check --kernel-timing all --config '127k x 47'" timeout -k 10 900 bash tools/sweep_env.sh "X=1" "FESOM2_NT=0" "FESOM2_NT=0 FESOM2_TILE_REV=2" "FESOM2_NT=2" "FESOM2_NT=4" "FESOM2_B3H_NT=0" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_nt_127k.txt
