set -o pipefail
mkdir -p gpurun_out
export FESOM2_LIB_NAME=libfesom2-accelerate.so
ROUNDS=3 STEPS=50 BENCH_ARGS="--no-check --config '127k x 47'" timeout -k 10 600 bash tools/sweep_env.sh "X=1 | --kernel-timing all" "X=1 | --kernel-timing dominant" "X=1 | --kernel-timing none" "X=1 | --kernel-timing none --graph" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_timing_127k.txt
ROUNDS=2 STEPS=20 BENCH_ARGS="--no-check" timeout -k 10 600 bash tools/sweep_env.sh "X=1 | --kernel-timing all" "X=1 | --kernel-timing dominant" "X=1 | --kernel-timing none" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_timing_1p2m.txt
export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_127k_none -o kt -- python3 bench.py --config "127k x 47" --no-cpu-baseline --no-check --steps 20 --kernel-timing none > gpurun_out/kt_127k_none.json 2> gpurun_out/kt_127k_none.err || exit 1
python3 tools/trace_gaps.py gpurun_out/kt_127k_none --last 60 > gpurun_out/kt_127k_none_gaps.txt || exit 1
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_127k_graph -o kt -- python3 bench.py --config "127k x 47" --no-cpu-baseline --no-check --steps 20 --graph > gpurun_out/kt_127k_graph.json 2> gpurun_out/kt_127k_graph.err || exit 1
python3 tools/trace_gaps.py gpurun_out/kt_127k_graph --last 60 > gpurun_out/kt_127k_graph_gaps.txt || exit 1
