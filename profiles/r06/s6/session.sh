#!/bin/bash
# round 6 session 6: A/B of the cluster unions + tracer groups with ONE set of field buffers for every
# variant (tools/ab_inproc.py; duplicate variants as the control), product and tuning builds
set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_inproc.py --config '127k x 47' --tracers 6 --rounds 21 --burst 20 \
    union= off=FESOM2_P1V_UNION=0 union_b= off_b=FESOM2_P1V_UNION=0 > gpurun_out/s6_ab_127k6.txt 2>&1
timeout -k 10 300 python -u tools/ab_inproc.py --config '127k x 47' --tracers 1 --rounds 21 --burst 80 \
    union= off=FESOM2_P1V_UNION=0 union_b= off_b=FESOM2_P1V_UNION=0 > gpurun_out/s6_ab_127k1.txt 2>&1
echo "product ab done"
FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so timeout -k 10 300 python -u tools/ab_inproc.py --config '127k x 47' \
    --tracers 6 --rounds 21 --burst 20 off=FESOM2_P1V_UNION=0 union= u_tg6=FESOM2_TRACER_GROUP=6 \
    off_tg3=FESOM2_P1V_UNION=0,FESOM2_TRACER_GROUP=3 u_tg2=FESOM2_TRACER_GROUP=2 u_cap16=FESOM2_P1V_UNION_MAX=16 \
    u_cap24=FESOM2_P1V_UNION_MAX=24 off_rp=FESOM2_P1V_UNION=0,FESOM2_ROWPAIR=1 > gpurun_out/s6_ab_127k6_parts.txt 2>&1
echo "tuning ab done"
