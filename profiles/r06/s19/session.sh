#!/bin/bash
# round 6 session 19 (tuning build): the union cap on Delaunay meshes at 127k x 47 (6 tracers)
set -eo pipefail
export TMPDIR=/tmp
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
for mesh in delaunay-hilbert delaunay; do
  timeout -k 10 400 python -u tools/ab_inproc.py --config '127k x 47' --mesh $mesh --tracers 6 --rounds 15 --burst 20 \
      base= c16=FESOM2_P1V_UNION_MAX=16 c24=FESOM2_P1V_UNION_MAX=24 c28=FESOM2_P1V_UNION_MAX=28 \
      c32=FESOM2_P1V_UNION_MAX=32 base_b= > gpurun_out/s19_ab_${mesh}_6.txt 2>&1
done
echo "ab done"
