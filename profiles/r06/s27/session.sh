#!/bin/bash
# round 6 session 27 (tuning build): p1v's vertical-tail loads (del_ttf_advvert, hnode, hnode_new,
# area) issued right after phase 1 instead of after the last barrier (FESOM2_P1V_EARLY, OPT 2048):
# union forms 74 VGPRs (6 waves/SIMD) against 62; large-partition stash form 76 (E=1) or held to 8
# waves with 60 B of spills (E=2)
set -eo pipefail
export TMPDIR=/tmp
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
for tr in 6 1; do
  timeout -k 10 400 python -u tools/ab_inproc.py --config '127k x 47' --tracers $tr --rounds 15 --burst 20 \
      base= early=FESOM2_P1V_EARLY=1 base_b= > gpurun_out/s27_ab_127k_${tr}.txt 2>&1
  echo "127k $tr done"
done
timeout -k 10 500 python -u tools/ab_inproc.py --config '1.2M x 80' --tracers 6 --rounds 7 --burst 4 \
    base= e1=FESOM2_P1V_EARLY=1 e2=FESOM2_P1V_EARLY=2 base_b= > gpurun_out/s27_ab_1p2M_6.txt 2>&1
echo "1.2M done"
