set -o pipefail
mkdir -p gpurun_out
ROUNDS=2 STEPS=20 BENCH_ARGS="--no-check --kernel-timing all --path reference-plain" timeout -k 10 900 bash tools/sweep_env.sh "X=1" "FESOM2_C_BATCH=2" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_cbatch_refplain_1p2m.txt
ROUNDS=2 STEPS=30 BENCH_ARGS="--no-check --kernel-timing all --path reference-plain --config '127k x 47'" timeout -k 10 600 bash tools/sweep_env.sh "X=1" "FESOM2_C_BATCH=2" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_cbatch_refplain_127k.txt
FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so FESOM2_C_BATCH=2 timeout -k 10 300 python bench.py --path reference-plain --no-cpu-baseline --steps 5 > gpurun_out/r03_cbatch_plain_check.json 2> gpurun_out/r03_cbatch_plain_check.err || exit 1
