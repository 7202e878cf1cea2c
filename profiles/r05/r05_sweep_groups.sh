#!/bin/bash
# Round 5: block sizes of the large-partition plans again, now that the stash form runs at 8
# waves/SIMD (tuning build; an explicit column count needs the row pairs, the stash and the internal
# edges switched on by hand: FESOM2_ROWPAIR / FESOM2_P1V_STASH / FESOM2_P1V_B3H).
set -eo pipefail
export TMPDIR=/tmp
RP="FESOM2_ROWPAIR=1 FESOM2_P1V_STASH=1 FESOM2_P1V_B3H=1"
ROUNDS=3 STEPS=20 BENCH_ARGS="--tracers 6" timeout -k 10 800 bash tools/sweep_env.sh \
    "FESOM2_BATCH_GROUP=0" "FESOM2_BATCH_GROUP=4 FESOM2_BATCH_PATCH=4096 $RP" \
    "FESOM2_BATCH_GROUP=8 FESOM2_BATCH_PATCH=4096 $RP" "FESOM2_BATCH_GROUP=10 FESOM2_BATCH_PATCH=4096 $RP"
cp gpurun_out/sweep.txt gpurun_out/r05j_sweep_batch_groups_6tr.txt
ROUNDS=3 STEPS=40 timeout -k 10 400 bash tools/sweep_env.sh \
    "FESOM2_GROUP=0" "FESOM2_GROUP=4 $RP" "FESOM2_GROUP=8 $RP"
cp gpurun_out/sweep.txt gpurun_out/r05j_sweep_groups_1tr.txt
