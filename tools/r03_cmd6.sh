set -o pipefail
bash tools/profile.sh r03a || exit 1
BENCH_ARGS="--config '127k x 47'" bash tools/profile.sh r03a_127k || exit 1
BENCH_ARGS="--tracers 6" bash tools/profile.sh r03a_6tr || exit 1
