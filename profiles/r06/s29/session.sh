#!/bin/bash
# round 6 session 29 (tuning build, timing only): what phase 2's gathers cost -- bit 6 packed b3h's
# plus/minus gathers, bit 2 the node kernel's edge gathers
set -eo pipefail
export TMPDIR=/tmp
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
V="base= a64=FESOM2_ABLATE=64 a4=FESOM2_ABLATE=4 base_b="
for tr in 6 1; do
  timeout -k 10 400 python -u tools/ab_inproc.py --config '127k x 47' --tracers $tr --rounds 15 --burst 20 $V \
      > gpurun_out/s29_ab_127k_${tr}.txt 2>&1
  echo "127k $tr done"
done
timeout -k 10 500 python -u tools/ab_inproc.py --config '1.2M x 80' --tracers 1 --rounds 9 --burst 10 $V \
    > gpurun_out/s29_ab_1p2M_1.txt 2>&1
echo "1.2M done"
