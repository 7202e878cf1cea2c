#!/bin/bash
# Round 5: the large-partition plan on BASELINE config 1 (127k x 47) now that its stash form fits 8
# waves/SIMD -- FESOM2_LARGE_CELLS=0 (5-column blocks in row pairs, the internal edges limited in p1v
# with their raw flux stashed in LDS; batched calls on 4096-node patches) and the internal edges
# alone (FESOM2_P1V_B3H=1) against the default, 1 and 6 tracers, product library, interleaved.
set -eo pipefail
export TMPDIR=/tmp
export FESOM2_LIB_NAME=libfesom2-accelerate.so
ROUNDS=3 STEPS=400 BENCH_ARGS="--config '127k x 47'" timeout -k 10 500 bash tools/sweep_env.sh \
    "FESOM2_LARGE_CELLS=33554432" "FESOM2_LARGE_CELLS=0" "FESOM2_P1V_B3H=1"
cp gpurun_out/sweep.txt gpurun_out/r05h_sweep_small_plan_1tr.txt
ROUNDS=3 STEPS=80 BENCH_ARGS="--config '127k x 47' --tracers 6" timeout -k 10 500 bash tools/sweep_env.sh \
    "FESOM2_LARGE_CELLS=33554432" "FESOM2_LARGE_CELLS=0" "FESOM2_P1V_B3H=1"
cp gpurun_out/sweep.txt gpurun_out/r05h_sweep_small_plan_6tr.txt
