set -o pipefail
mkdir -p gpurun_out
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
ROUNDS=2 STEPS=10 BENCH_ARGS="--no-check --tracers 6" timeout -k 10 900 bash tools/sweep_env.sh "FESOM2_TRACER_CHUNK=0" "FESOM2_TRACER_CHUNK=96" "FESOM2_TRACER_CHUNK=256" "FESOM2_TRACER_CHUNK=512" "FESOM2_TRACER_CHUNK=1024" || exit 1
cp gpurun_out/sweep.txt gpurun_out/r03_sweep_chunk_6tr.txt
FESOM2_TRACER_CHUNK=256 timeout -k 10 300 python bench.py --tracers 6 --no-cpu-baseline --steps 5 > gpurun_out/r03_chunk256_check.json 2> gpurun_out/r03_chunk256_check.err || exit 1
export TMPDIR=/tmp
for K in 0 256; do
FESOM2_TRACER_CHUNK=$K timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum \
    --output-format csv -d gpurun_out/pmc_chunk$K/rd -o rd -- python3 bench.py --no-cpu-baseline --no-check --steps 2 --warmup 1 --tracers 6 > /dev/null 2> gpurun_out/pmc_chunk$K.rd.err || exit 1
FESOM2_TRACER_CHUNK=$K timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
    --output-format csv -d gpurun_out/pmc_chunk$K/wr -o wr -- python3 bench.py --no-cpu-baseline --no-check --steps 2 --warmup 1 --tracers 6 > /dev/null 2> gpurun_out/pmc_chunk$K.wr.err || exit 1
done
unset FESOM2_LIB_NAME
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_127k -o kt -- python3 bench.py --config "127k x 47" --no-cpu-baseline --no-check --steps 20 > gpurun_out/kt_127k.json 2> gpurun_out/kt_127k.err || exit 1
python3 tools/trace_gaps.py gpurun_out/kt_127k --last 60 > gpurun_out/kt_127k_gaps.txt || exit 1
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_1p2m -o kt -- python3 bench.py --no-cpu-baseline --no-check --steps 20 > gpurun_out/kt_1p2m.json 2> gpurun_out/kt_1p2m.err || exit 1
python3 tools/trace_gaps.py gpurun_out/kt_1p2m --last 60 > gpurun_out/kt_1p2m_gaps.txt || exit 1
