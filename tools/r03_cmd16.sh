set -o pipefail
mkdir -p gpurun_out
ROUNDS=2 STEPS=10 BENCH_ARGS="--no-check --kernel-timing all --tracers 6" timeout -k 10 900 bash tools/sweep_env.sh "X=1" "FESOM2_PATCH=1024" "FESOM2_TRACER_CHUNK=8" "FESOM2_TRACER_CHUNK=16" "FESOM2_TRACER_CHUNK=32" "FESOM2_PATCH=1024 FESOM2_TRACER_CHUNK=8" "FESOM2_PATCH=1024 FESOM2_TRACER_CHUNK=16" "FESOM2_PATCH=1024 FESOM2_TRACER_CHUNK=32" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_chunk_small_6tr.txt
export TMPDIR=/tmp FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
for cfg in "X=1|6" "FESOM2_TRACER_CHUNK=256|6" "FESOM2_PATCH=1024|6" "X=1|1"; do
  envs=${cfg%%|*}; ntr=${cfg#*|}; tag=$(echo "$envs" | tr '= ' '__')_$ntr
  env $envs timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/tcc_$tag -o tcc -- python3 bench.py --no-cpu-baseline --no-check --steps 2 --warmup 1 --tracers $ntr > /dev/null 2> gpurun_out/tcc_$tag.err || exit 1
done
