set -o pipefail
mkdir -p gpurun_out
ROUNDS=3 STEPS=50 BENCH_ARGS="--no-check --kernel-timing none --config '127k x 47'" timeout -k 10 800 bash tools/sweep_env.sh "X=1" "FESOM2_XCD=0" "FESOM2_P2H_FUSE=1" "FESOM2_P1V_B3H=1" "FESOM2_XCD=0 FESOM2_P1V_B3H=1" "FESOM2_PATCH=4096" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_127k_knobs.txt
FESOM2_LIB_NAME=libfesom2-accelerate.so timeout -k 10 300 python bench.py --config "127k x 47" --no-cpu-baseline > gpurun_out/r03_127k_dominant.json 2> gpurun_out/r03_127k_dominant.err || exit 1
