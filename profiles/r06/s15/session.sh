#!/bin/bash
# round 6 session 15 (tuning build, its launch-time knobs now re-read at every launch): tile orders
# of the batched union plan at 6 x 127k x 47 -- tracer groups, tracer-slowest kernels -- and the
# gather ablations under unions (timing only), shared buffers
set -eo pipefail
export TMPDIR=/tmp
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
timeout -k 10 400 python -u tools/ab_inproc.py --config '127k x 47' --tracers 6 --rounds 15 --burst 20 \
    base= tg2=FESOM2_TRACER_GROUP=2 tg3=FESOM2_TRACER_GROUP=3 tm3=FESOM2_TRACER_MAJOR=3 tm7=FESOM2_TRACER_MAJOR=7 \
    tm0=FESOM2_TRACER_MAJOR=0 abl1=FESOM2_ABLATE=1 abl2=FESOM2_ABLATE=2 abl4=FESOM2_ABLATE=4 base_b= \
    > gpurun_out/s15_ab_127k6.txt 2>&1
echo "ab done"
timeout -k 10 600 python -u tools/ab_inproc.py --config '1.2M x 80' --tracers 6 --rounds 7 --burst 4 \
    base= tg2=FESOM2_TRACER_GROUP=2 tg3=FESOM2_TRACER_GROUP=3 base_b= > gpurun_out/s15_ab_1p2M6.txt 2>&1
echo "ab2 done"
