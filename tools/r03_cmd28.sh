set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r03_gputests_vl.log 2>&1 || exit 1
export FESOM2_LIB_NAME=libfesom2-accelerate.so
ROUNDS=2 STEPS=30 BENCH_ARGS="--no-check --kernel-timing all --config '127k x 47'" timeout -k 10 600 bash tools/sweep_env.sh "X=1 | --vlimit 1" "X=1 | --vlimit 2" "X=1 | --vlimit 3" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_vlimit_127k.txt
timeout -k 10 300 python bench.py --config "127k x 47" --vlimit 2 --no-cpu-baseline > gpurun_out/r03_vl2_127k_check.json 2> gpurun_out/r03_vl2_127k_check.err || exit 1
