#!/bin/bash
# Round 5: 12- and 16-column blocks of the large-partition plans (tuning build), after the memory
# counters (profiles/r05/mem/) showed every CU's L1 stalled on pending misses: a 12-column block
# (480 threads = 8 waves; 4 blocks fill the CU's 32 wave slots) shares more neighbour columns inside
# one block -- fewer L1 -> L2 requests per byte?  16 columns = 10 waves (3 blocks, 30 slots).
set -eo pipefail
export TMPDIR=/tmp
RP="FESOM2_ROWPAIR=1 FESOM2_P1V_STASH=1 FESOM2_P1V_B3H=1"
FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so FESOM2_BATCH_GROUP=12 FESOM2_BATCH_PATCH=4096 FESOM2_ROWPAIR=1 \
    FESOM2_P1V_STASH=1 FESOM2_P1V_B3H=1 timeout -k 10 300 python bench.py --no-cpu-baseline --extras none --tracers 6 \
    > gpurun_out/r05t_group12_6tr_check.json 2> gpurun_out/r05t_group12_6tr_check.err
ROUNDS=3 STEPS=20 BENCH_ARGS="--tracers 6" timeout -k 10 800 bash tools/sweep_env.sh \
    "FESOM2_BATCH_GROUP=0" "FESOM2_BATCH_GROUP=12 FESOM2_BATCH_PATCH=4096 $RP" \
    "FESOM2_BATCH_GROUP=16 FESOM2_BATCH_PATCH=4096 $RP"
cp gpurun_out/sweep.txt gpurun_out/r05t_sweep_batch_groups12_6tr.txt
ROUNDS=3 STEPS=40 timeout -k 10 400 bash tools/sweep_env.sh "FESOM2_GROUP=0" "FESOM2_GROUP=12 $RP"
cp gpurun_out/sweep.txt gpurun_out/r05t_sweep_groups12_1tr.txt
echo "sweeps done"
