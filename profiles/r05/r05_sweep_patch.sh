#!/bin/bash
# Round 5: patch sizes of the large-partition plans with the stash form at 8 waves/SIMD (tuning
# build): the batched plan (FESOM2_BATCH_PATCH, 6 x 1.2M x 80) and the single-tracer one
# (FESOM2_PATCH, 1.2M x 80), interleaved rounds.
set -eo pipefail
export TMPDIR=/tmp
ROUNDS=3 STEPS=20 BENCH_ARGS="--tracers 6" timeout -k 10 700 bash tools/sweep_env.sh \
    "FESOM2_BATCH_PATCH=2048" "FESOM2_BATCH_PATCH=4096" "FESOM2_BATCH_PATCH=8192" "FESOM2_BATCH_PATCH=16384"
cp gpurun_out/sweep.txt gpurun_out/r05g_sweep_batch_patch_6tr.txt
ROUNDS=3 STEPS=40 timeout -k 10 400 bash tools/sweep_env.sh \
    "FESOM2_PATCH=8192" "FESOM2_PATCH=16384" "FESOM2_PATCH=32768"
cp gpurun_out/sweep.txt gpurun_out/r05g_sweep_patch_1tr.txt
