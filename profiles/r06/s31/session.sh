#!/bin/bash
# round 6 session 31 (tuning build): p1v's plus/minus as cache-allocating stores (FESOM2_P1V_PMPLAIN,
# OPT 8192) so that b3h can read them from the Infinity Cache; with and without the cache pass order
set -eo pipefail
export TMPDIR=/tmp
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
V="base= pm=FESOM2_P1V_PMPLAIN=1 co=FESOM2_CACHE_ORDER=1 pm_co=FESOM2_P1V_PMPLAIN=1,FESOM2_CACHE_ORDER=1 base_b= pm_b=FESOM2_P1V_PMPLAIN=1"
for tr in 1 6; do
  timeout -k 10 400 python -u tools/ab_inproc.py --config '127k x 47' --tracers $tr --rounds 15 --burst 20 $V \
      > gpurun_out/s31_ab_127k_${tr}.txt 2>&1
  echo "127k $tr done"
done
