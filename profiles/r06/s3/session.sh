#!/bin/bash
# round 6 session 3: in-process interleaved A/B (tools/ab_inproc.py) of the capped cluster-union p1v
# with row-pair blocks and of tracer-group tile orders at 127k x 47
set -eo pipefail
export TMPDIR=/tmp
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
U="FESOM2_P1V_UNION=2,FESOM2_ROWPAIR=1"
timeout -k 10 300 python -u tools/ab_inproc.py --config '127k x 47' --tracers 6 --rounds 15 --burst 10 base= \
    u2rp=$U u2rp16=$U,FESOM2_P1V_UNION_MAX=16 u2rp18=$U,FESOM2_P1V_UNION_MAX=18 u2rp20=$U,FESOM2_P1V_UNION_MAX=20 \
    u2rp22=$U,FESOM2_P1V_UNION_MAX=22 rp=FESOM2_ROWPAIR=1 > gpurun_out/s3_ab_127k6_union.txt 2>&1
echo "ab1 done"
timeout -k 10 300 python -u tools/ab_inproc.py --config '127k x 47' --tracers 6 --rounds 15 --burst 10 base= \
    tg2=FESOM2_TRACER_GROUP=2 tg3=FESOM2_TRACER_GROUP=3 u2rp20tg3=$U,FESOM2_P1V_UNION_MAX=20,FESOM2_TRACER_GROUP=3 \
    u2rp20tg2=$U,FESOM2_P1V_UNION_MAX=20,FESOM2_TRACER_GROUP=2 > gpurun_out/s3_ab_127k6_tg.txt 2>&1
echo "ab2 done"
timeout -k 10 300 python -u tools/ab_inproc.py --config '127k x 47' --tracers 1 --rounds 15 --burst 40 base= \
    u2rp16=$U,FESOM2_P1V_UNION_MAX=16 u2rp18=$U,FESOM2_P1V_UNION_MAX=18 u2rp20=$U,FESOM2_P1V_UNION_MAX=20 \
    u2=FESOM2_P1V_UNION=2 > gpurun_out/s3_ab_127k1_union.txt 2>&1
echo "ab3 done"
