#!/bin/bash
# round 6 session 11 (tuning build): the cluster union in two halves of the levels on the large
# plan -- exactness, then shared-buffer A/B at 6 x 1.2M x 80 and 1.2M x 80
set -eo pipefail
export TMPDIR=/tmp
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_tuning.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "level_halves or cluster_union" > gpurun_out/s11_tests.log 2>&1
echo "tests done"
H="FESOM2_P1V_UNION=1,FESOM2_P1V_UNION_HALF"
timeout -k 10 900 python -u tools/ab_inproc.py --config '1.2M x 80' --tracers 6 --rounds 9 --burst 4 \
    base= h1c17=$H=1,FESOM2_P1V_UNION_MAX=17 h2c17=$H=2,FESOM2_P1V_UNION_MAX=17 h1c18=$H=1,FESOM2_P1V_UNION_MAX=18 \
    h1c14=$H=1,FESOM2_P1V_UNION_MAX=14 base_b= > gpurun_out/s11_ab_1p2M6.txt 2>&1
echo "ab 1p2M6 done"
timeout -k 10 600 python -u tools/ab_inproc.py --config '1.2M x 80' --tracers 1 --rounds 15 --burst 10 \
    base= h1c17=$H=1,FESOM2_P1V_UNION_MAX=17 h2c17=$H=2,FESOM2_P1V_UNION_MAX=17 base_b= > gpurun_out/s11_ab_1p2M1.txt 2>&1
echo "ab 1p2M1 done"
