set -o pipefail
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
ROUNDS=2 STEPS=10 BENCH_ARGS="--no-check --tracers 6" timeout -k 10 900 bash tools/sweep_env.sh "FESOM2_TRACER_CHUNK=0" "FESOM2_TRACER_CHUNK=64" "FESOM2_TRACER_CHUNK=256" "FESOM2_TRACER_CHUNK=1024" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_chunk_6tr.txt
FESOM2_TRACER_CHUNK=256 timeout -k 10 300 python bench.py --tracers 6 --no-cpu-baseline --steps 5 > gpurun_out/r03_chunk256_check.json 2> gpurun_out/r03_chunk256_check.err || exit 1
unset FESOM2_LIB_NAME
timeout -k 10 300 python bench.py > gpurun_out/r03_default2.json 2> gpurun_out/r03_default2.err || exit 1
