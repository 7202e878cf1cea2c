#!/bin/bash
# round 6 session 5: the product build with cluster unions + tracer groups on small partitions --
# full GPU suite, the tuning variants' tests, in-process A/B against FESOM2_P1V_UNION=0 (with
# duplicate variants as a placement control), and the default bench with every leg
set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 600 --timeout-method thread \
    > gpurun_out/s5_gputests.log 2>&1
echo "gpu tests done"
FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so timeout -k 10 300 python -u -m pytest tests/test_gpu_tuning.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -k "cluster_union or tracer_group" > gpurun_out/s5_tuning_tests.log 2>&1
echo "tuning tests done"
timeout -k 10 300 python -u tools/ab_inproc.py --config '127k x 47' --tracers 6 --rounds 21 --burst 20 \
    union= off=FESOM2_P1V_UNION=0 union_b= off_b=FESOM2_P1V_UNION=0 > gpurun_out/s5_ab_127k6.txt 2>&1
timeout -k 10 300 python -u tools/ab_inproc.py --config '127k x 47' --tracers 1 --rounds 21 --burst 80 \
    union= off=FESOM2_P1V_UNION=0 union_b= off_b=FESOM2_P1V_UNION=0 > gpurun_out/s5_ab_127k1.txt 2>&1
echo "ab done"
timeout -k 10 900 python -u bench.py > gpurun_out/s5_bench.json 2> gpurun_out/s5_bench.err
echo "bench done"
