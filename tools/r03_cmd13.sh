set -o pipefail
mkdir -p gpurun_out
# batched p1v (6 tracers) vs single under the timing-only ablations (results wrong: --no-check)
ROUNDS=2 STEPS=10 BENCH_ARGS="--no-check --kernel-timing all --tracers 6" timeout -k 10 700 bash tools/sweep_env.sh "X=1" "FESOM2_ABLATE=1" "FESOM2_ABLATE=2" "FESOM2_ABLATE=3" "FESOM2_TRACER_MAJOR=3" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_ablate_6tr.txt
ROUNDS=2 STEPS=20 BENCH_ARGS="--no-check --kernel-timing all" timeout -k 10 500 bash tools/sweep_env.sh "X=1" "FESOM2_ABLATE=1" "FESOM2_ABLATE=2" "FESOM2_ABLATE=3" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_ablate_1tr.txt
