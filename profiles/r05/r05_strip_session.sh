#!/bin/bash
# Round-5 GPU session for the batched p1v (config 3): strip orders inside the batched plan's
# patches (tuning build, FESOM2_BATCH_STRIP).  Every step has its own time bound; the first failure
# ends the session (set -e).
#   1. parity of the strip orders (tests/test_gpu_tuning.py -k strip)
#   2. a full-size exact check of 6 x 1.2M x 80 with strips of 18
#   3. interleaved A/B of strip widths at 6 x 1.2M x 80 and 6 x 127k x 47 (tools/sweep_env.sh)
#   4. PMC L2-miss reads per variant (tools/pmc_batch_ablate.sh)
# usage: bash tools/r05_strip_session.sh [a|b]   (a: steps 1-3 at 1.2M x 80; b: the 127k sweep and step 4)
set -eo pipefail
part=${1:-a}
export TMPDIR=/tmp
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
mkdir -p gpurun_out
if [ "$part" = a ]; then
timeout -k 10 300 python -u -m pytest tests/test_gpu_tuning.py -m gpu -k strip -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/r05b_strip_tests.log 2>&1
echo "strip tests ok"
FESOM2_BATCH_STRIP=18 timeout -k 10 300 python bench.py --tracers 6 --no-cpu-baseline --extras none \
    > gpurun_out/r05b_strip18_6tr_check.json 2> gpurun_out/r05b_strip18_6tr_check.err
echo "full-size check ok"
ROUNDS=3 STEPS=20 BENCH_ARGS="--tracers 6" timeout -k 10 900 bash tools/sweep_env.sh \
    "FESOM2_BATCH_STRIP=0" "FESOM2_BATCH_STRIP=12" "FESOM2_BATCH_STRIP=18" "FESOM2_BATCH_STRIP=24" \
    "FESOM2_BATCH_STRIP=36"
cp gpurun_out/sweep.txt gpurun_out/r05b_sweep_strip_6tr_1p2M.txt
echo "sweep 1.2M done"
else
ROUNDS=3 STEPS=100 BENCH_ARGS="--tracers 6 --config '127k x 47'" timeout -k 10 600 bash tools/sweep_env.sh \
    "FESOM2_BATCH_STRIP=0" "FESOM2_BATCH_STRIP=16" "FESOM2_BATCH_STRIP=32"
cp gpurun_out/sweep.txt gpurun_out/r05b_sweep_strip_6tr_127k.txt
echo "sweep 127k done"
timeout -k 10 900 bash tools/pmc_batch_ablate.sh r05b default strip18 strip24 nocluster noedge
echo "pmc done"
fi
