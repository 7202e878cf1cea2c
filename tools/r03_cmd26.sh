set -o pipefail
mkdir -p gpurun_out
ROUNDS=2 STEPS=20 BENCH_ARGS="--no-check --kernel-timing all" timeout -k 10 900 bash tools/sweep_env.sh "X=1 | --path reference" "FESOM2_C_BATCH=2 | --path reference" "X=1 | --path fused" "FESOM2_P2_BATCH=2 | --path fused" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_cbatch_1p2m.txt
ROUNDS=2 STEPS=30 BENCH_ARGS="--no-check --kernel-timing all --config '127k x 47'" timeout -k 10 600 bash tools/sweep_env.sh "X=1 | --path reference" "FESOM2_C_BATCH=2 | --path reference" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_cbatch_127k.txt
FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so FESOM2_C_BATCH=2 timeout -k 10 300 python bench.py --path reference --no-cpu-baseline --steps 5 > gpurun_out/r03_cbatch_check.json 2> gpurun_out/r03_cbatch_check.err || exit 1
FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so FESOM2_P2_BATCH=2 timeout -k 10 300 python bench.py --path fused --no-cpu-baseline --steps 5 > gpurun_out/r03_p2batch_check.json 2> gpurun_out/r03_p2batch_check.err || exit 1
