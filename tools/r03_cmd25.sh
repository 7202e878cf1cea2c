set -o pipefail
mkdir -p gpurun_out
BENCH_ARGS="--config '127k x 47'" timeout -k 10 600 bash tools/profile.sh r03c_127k || exit 1
timeout -k 10 600 bash tools/profile.sh r03c || exit 1
