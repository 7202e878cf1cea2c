#!/bin/bash
# round 6 session 22 (tuning build): larger p1v blocks for the cluster unions at 127k x 47 --
# G columns in R rows (FESOM2_GROUP / FESOM2_BATCH_GROUP, FESOM2_ROWPAIR), the union cap raised to
# hold the block's whole union; patches pinned at 16384 nodes (an explicit column count would
# otherwise switch them to 4096)
set -eo pipefail
export TMPDIR=/tmp
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
P=FESOM2_PATCH=16384,FESOM2_BATCH_PATCH=16384
v() { echo "$1=FESOM2_GROUP=$2,FESOM2_BATCH_GROUP=$2,FESOM2_ROWPAIR=$3,FESOM2_P1V_UNION_MAX=$4,$P"; }
for tr in 6 1; do
  timeout -k 10 500 python -u tools/ab_inproc.py --config '127k x 47' --tracers $tr --rounds 15 --burst 20 \
      base= basep=$P "$(v g12r2 12 2 30)" "$(v g12r3 12 3 28)" "$(v g16r4 16 4 34)" "$(v g16r2 16 2 38)" \
      "$(v g20r4 20 4 40)" base_b= > gpurun_out/s22_ab_127k_${tr}.txt 2>&1
  echo "tracers $tr done"
done
