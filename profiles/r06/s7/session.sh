#!/bin/bash
# round 6 session 7: union plans with b3h / phase 2 in the patches' plain order -- parity on the small
# meshes, then the shared-buffer A/B against FESOM2_P1V_UNION=0 (duplicates as the control)
set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batched.py tests/test_gpu_halo.py \
    tests/test_gpu_graph.py tests/test_gpu_unstructured.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/s7_gputests.log 2>&1
echo "tests done"
timeout -k 10 300 python -u tools/ab_inproc.py --config '127k x 47' --tracers 6 --rounds 21 --burst 20 \
    union= off=FESOM2_P1V_UNION=0 union_b= off_b=FESOM2_P1V_UNION=0 > gpurun_out/s7_ab_127k6.txt 2>&1
timeout -k 10 300 python -u tools/ab_inproc.py --config '127k x 47' --tracers 1 --rounds 21 --burst 80 \
    union= off=FESOM2_P1V_UNION=0 union_b= off_b=FESOM2_P1V_UNION=0 > gpurun_out/s7_ab_127k1.txt 2>&1
echo "ab done"
