#!/bin/bash
# round 6 session 26 (tuning build, timing only -- ablated results are wrong): what p1v's loads cost
# -- bit 3 the second fct_adf_v load, bit 4 the vertical tail's loads, bit 5 the union DMA, bit 1
# the edge gathers (reference)
set -eo pipefail
export TMPDIR=/tmp
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
V="base= a8=FESOM2_ABLATE=8 a16=FESOM2_ABLATE=16 a32=FESOM2_ABLATE=32 a2=FESOM2_ABLATE=2 base_b="
for tr in 6 1; do
  timeout -k 10 400 python -u tools/ab_inproc.py --config '127k x 47' --tracers $tr --rounds 15 --burst 20 $V \
      > gpurun_out/s26_ab_127k_${tr}.txt 2>&1
  echo "127k $tr done"
done
timeout -k 10 500 python -u tools/ab_inproc.py --config '1.2M x 80' --tracers 1 --rounds 9 --burst 10 $V \
    > gpurun_out/s26_ab_1p2M_1.txt 2>&1
echo "1.2M done"
