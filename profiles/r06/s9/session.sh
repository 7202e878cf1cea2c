#!/bin/bash
# round 6 session 9 (tuning build): p1v blocks of one column group for two tracers (FESOM2_P1V_TP=2)
# -- exactness, then shared-buffer A/B at 6 x 1.2M x 80 (config 3) and 6 x 127k x 47 without unions
set -eo pipefail
export TMPDIR=/tmp
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_tuning.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "tracer_halves" > gpurun_out/s9_tests.log 2>&1
echo "tests done"
timeout -k 10 600 python -u tools/ab_inproc.py --config '1.2M x 80' --tracers 6 --rounds 9 --burst 4 \
    base= tp2=FESOM2_P1V_TP=2 tp2w7=FESOM2_P1V_TP=2,FESOM2_P1V_TP_W8=0 base_b= > gpurun_out/s9_ab_1p2M6.txt 2>&1
echo "ab 1p2M6 done"
timeout -k 10 300 python -u tools/ab_inproc.py --config '127k x 47' --tracers 6 --rounds 21 --burst 20 \
    off=FESOM2_P1V_UNION=0 off_tp2=FESOM2_P1V_UNION=0,FESOM2_P1V_TP=2 union= off_b=FESOM2_P1V_UNION=0 \
    > gpurun_out/s9_ab_127k6.txt 2>&1
echo "ab 127k6 done"
