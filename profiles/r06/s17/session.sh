#!/bin/bash
# round 6 session 17 (tuning build): b1h edge gathers per round trip in the union forms
set -eo pipefail
export TMPDIR=/tmp
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_tuning.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "union_edge_batches" > gpurun_out/s17_tests.log 2>&1
echo "tests done"
timeout -k 10 300 python -u tools/ab_inproc.py --config '127k x 47' --tracers 6 --rounds 15 --burst 20 \
    base= eb3=FESOM2_P1V_UNION_EB=3 eb4=FESOM2_P1V_UNION_EB=4 base_b= > gpurun_out/s17_ab_127k6.txt 2>&1
timeout -k 10 300 python -u tools/ab_inproc.py --config '127k x 47' --tracers 1 --rounds 15 --burst 80 \
    base= eb3=FESOM2_P1V_UNION_EB=3 eb4=FESOM2_P1V_UNION_EB=4 base_b= > gpurun_out/s17_ab_127k1.txt 2>&1
echo "ab done"
