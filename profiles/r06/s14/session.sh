#!/bin/bash
# round 6 session 14 (tuning build): the batched union plan's reuse distance at 6 x 127k x 47 --
# smaller patches for the batched plan, tracer-slowest p1 tiles, tracer groups (shared buffers)
set -eo pipefail
export TMPDIR=/tmp
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
timeout -k 10 400 python -u tools/ab_inproc.py --config '127k x 47' --tracers 6 --rounds 15 --burst 20 \
    base= bp1024=FESOM2_BATCH_PATCH=1024 bp2048=FESOM2_BATCH_PATCH=2048 bp4096=FESOM2_BATCH_PATCH=4096 \
    bp8192=FESOM2_BATCH_PATCH=8192 tm1=FESOM2_TRACER_MAJOR=3 tg2=FESOM2_TRACER_GROUP=2 \
    bp4096tg2=FESOM2_BATCH_PATCH=4096,FESOM2_TRACER_GROUP=2 bp2048tg3=FESOM2_BATCH_PATCH=2048,FESOM2_TRACER_GROUP=3 \
    base_b= > gpurun_out/s14_ab_127k6.txt 2>&1
echo "ab done"
