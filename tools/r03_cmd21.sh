set -o pipefail
mkdir -p gpurun_out
ROUNDS=3 STEPS=50 BENCH_ARGS="--no-check --kernel-timing none --config '127k x 47'" timeout -k 10 800 bash tools/sweep_env.sh "X=1" "FESOM2_TILE_REV=2" "FESOM2_TILE_REV=4" "FESOM2_TILE_REV=6" "FESOM2_TILE_REV=3" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_rev_127k.txt
ROUNDS=2 STEPS=20 BENCH_ARGS="--no-check --kernel-timing all" timeout -k 10 600 bash tools/sweep_env.sh "X=1" "FESOM2_TILE_REV=2" "FESOM2_TILE_REV=4" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_rev_1p2m.txt
FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so FESOM2_TILE_REV=6 timeout -k 10 300 python bench.py --config "127k x 47" --no-cpu-baseline --steps 5 --tracers 2 > gpurun_out/r03_rev6_check.json 2> gpurun_out/r03_rev6_check.err || exit 1
