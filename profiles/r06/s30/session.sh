#!/bin/bash
# round 6 session 30 (tuning build): packed b3h with each block's endpoint union staged in LDS
# (FESOM2_B3H_UNION, k_b3h_pu): exactness first, then the A/B
set -o pipefail
export TMPDIR=/tmp
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_tuning.py -m gpu -v -k endpoint_union --timeout 120 \
    --timeout-method thread > gpurun_out/s30_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
V="base= u24=FESOM2_B3H_UNION=1 u16=FESOM2_B3H_UNION=1,FESOM2_B3H_UNION_KB=16 base_b= u24_b=FESOM2_B3H_UNION=1"
for tr in 6 1; do
  timeout -k 10 400 python -u tools/ab_inproc.py --config '127k x 47' --tracers $tr --rounds 15 --burst 20 $V \
      > gpurun_out/s30_ab_127k_${tr}.txt 2>&1 || exit $?
  echo "127k $tr done"
done
for tr in 1 6; do
  timeout -k 10 500 python -u tools/ab_inproc.py --config '1.2M x 80' --tracers $tr --rounds 7 --burst 5 $V \
      > gpurun_out/s30_ab_1p2M_${tr}.txt 2>&1 || exit $?
  echo "1.2M $tr done"
done
