#!/bin/bash
# round 6 session 28 (tuning build): p1v's vertical-tail loads staged into LDS by DMA right after
# phase 1 (FESOM2_P1V_STAGE, OPT 4096, 64 VGPRs): exactness first, then the A/B at 127k x 47
set -o pipefail
export TMPDIR=/tmp
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_tuning.py -m gpu -v -k staged_tail --timeout 120 \
    --timeout-method thread > gpurun_out/s28_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
for tr in 6 1; do
  timeout -k 10 400 python -u tools/ab_inproc.py --config '127k x 47' --tracers $tr --rounds 15 --burst 20 \
      base= stage=FESOM2_P1V_STAGE=1 base_b= stage_b=FESOM2_P1V_STAGE=1 > gpurun_out/s28_ab_127k_${tr}.txt 2>&1 || exit $?
  echo "127k $tr done"
done
