set -o pipefail
mkdir -p gpurun_out
ROUNDS=2 STEPS=10 BENCH_ARGS="--no-check --kernel-timing all --tracers 6" timeout -k 10 900 bash tools/sweep_env.sh "X=1" "FESOM2_P1V_WAVES=8" "FESOM2_P1V_WAVES=7" "FESOM2_P1V_EARLY=12" "FESOM2_TRACER_MAJOR=6" "FESOM2_TRACER_MAJOR=0" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_waves_6tr.txt
