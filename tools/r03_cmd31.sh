set -o pipefail
mkdir -p gpurun_out
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
FESOM2_P2H_BATCH=6 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/r03_p2h6_check.json 2> gpurun_out/r03_p2h6_check.err || exit 1
FESOM2_P2H_BATCH=6 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --config "127k x 47" > gpurun_out/r03_p2h6_127k_check.json 2> gpurun_out/r03_p2h6_127k_check.err || exit 1
ROUNDS=3 STEPS=20 BENCH_ARGS="--no-check --kernel-timing all" timeout -k 10 600 bash tools/sweep_env.sh "X=1" "FESOM2_P2H_BATCH=6" "FESOM2_P2H_BATCH=8" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_p2hbatch_1p2m.txt
ROUNDS=3 STEPS=50 BENCH_ARGS="--no-check --kernel-timing all --config '127k x 47'" timeout -k 10 600 bash tools/sweep_env.sh "X=1" "FESOM2_P2H_BATCH=6" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_p2hbatch_127k.txt
ROUNDS=1 STEPS=10 BENCH_ARGS="--no-check --kernel-timing all --tracers 6" timeout -k 10 600 bash tools/sweep_env.sh "X=1" "FESOM2_P2H_BATCH=6" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_p2hbatch_6tr.txt
