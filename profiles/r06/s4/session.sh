#!/bin/bash
# round 6 session 4: confirm the union + tracer-group combination (in-process interleaved A/B)
set -eo pipefail
export TMPDIR=/tmp
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
U="FESOM2_P1V_UNION=2,FESOM2_ROWPAIR=1"
timeout -k 10 400 python -u tools/ab_inproc.py --config '127k x 47' --tracers 6 --rounds 21 --burst 20 base= \
    tg3=FESOM2_TRACER_GROUP=3 u2rp20tg3=$U,FESOM2_P1V_UNION_MAX=20,FESOM2_TRACER_GROUP=3 \
    u2rp22tg3=$U,FESOM2_P1V_UNION_MAX=22,FESOM2_TRACER_GROUP=3 u2rp16tg3=$U,FESOM2_P1V_UNION_MAX=16,FESOM2_TRACER_GROUP=3 \
    u2rptg3=$U,FESOM2_TRACER_GROUP=3 u2rp20tg2=$U,FESOM2_P1V_UNION_MAX=20,FESOM2_TRACER_GROUP=2 \
    u2rp20=$U,FESOM2_P1V_UNION_MAX=20 > gpurun_out/s4_ab_127k6.txt 2>&1
echo "ab1 done"
timeout -k 10 400 python -u tools/ab_inproc.py --config '127k x 47' --tracers 1 --rounds 21 --burst 80 base= \
    u2rp20=$U,FESOM2_P1V_UNION_MAX=20 u2rp22=$U,FESOM2_P1V_UNION_MAX=22 u2rp16=$U,FESOM2_P1V_UNION_MAX=16 \
    > gpurun_out/s4_ab_127k1.txt 2>&1
echo "ab2 done"
timeout -k 10 600 python -u tools/ab_inproc.py --config '1.2M x 80' --tracers 6 --rounds 7 --burst 3 base= \
    tg3=FESOM2_TRACER_GROUP=3 tg2=FESOM2_TRACER_GROUP=2 > gpurun_out/s4_ab_1p2M6.txt 2>&1
echo "ab3 done"
