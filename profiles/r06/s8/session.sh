#!/bin/bash
# round 6 session 8 (tuning build): a batch's phase 2 one tracer at a time, and the block-internal
# edges limited in p1v on the union plan's row-pair blocks -- exactness, then shared-buffer A/B
set -eo pipefail
export TMPDIR=/tmp
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_tuning.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "per_tracer or cluster_union" > gpurun_out/s8_tests.log 2>&1
echo "tests done"
timeout -k 10 300 python -u tools/ab_inproc.py --config '127k x 47' --tracers 6 --rounds 21 --burst 20 \
    union= off=FESOM2_P1V_UNION=0 p2pt=FESOM2_P2_PER_TRACER=1 ib3h=FESOM2_P1V_B3H=1 \
    ib3h_p2pt=FESOM2_P1V_B3H=1,FESOM2_P2_PER_TRACER=1 union_b= > gpurun_out/s8_ab_127k6.txt 2>&1
timeout -k 10 300 python -u tools/ab_inproc.py --config '127k x 47' --tracers 1 --rounds 21 --burst 80 \
    union= off=FESOM2_P1V_UNION=0 ib3h=FESOM2_P1V_B3H=1 union_b= > gpurun_out/s8_ab_127k1.txt 2>&1
echo "ab done"
