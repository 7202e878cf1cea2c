#!/bin/bash
# round 6 session 18: the union plans on unstructured meshes (Delaunay, Hilbert and scattered numbering)
# at 127k x 47 -- plan statistics + full-size exactness (tuning build, bench check), then the product's
# shared-buffer A/B against FESOM2_P1V_UNION=0
set -eo pipefail
export TMPDIR=/tmp
for mesh in delaunay-hilbert delaunay; do
  for tr in 1 6; do
    FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so FESOM2_PLAN_STATS=1 timeout -k 10 300 python bench.py --no-cpu-baseline \
        --extras none --steps 3 --warmup 1 --config '127k x 47' --mesh $mesh --tracers $tr \
        > gpurun_out/s18_check_${mesh}_${tr}.json 2> gpurun_out/s18_check_${mesh}_${tr}.err
  done
done
echo "checks done"
for mesh in delaunay-hilbert delaunay; do
  timeout -k 10 400 python -u tools/ab_inproc.py --config '127k x 47' --mesh $mesh --tracers 6 --rounds 15 --burst 20 \
      union= off=FESOM2_P1V_UNION=0 union_b= off_b=FESOM2_P1V_UNION=0 > gpurun_out/s18_ab_${mesh}_6.txt 2>&1
  timeout -k 10 400 python -u tools/ab_inproc.py --config '127k x 47' --mesh $mesh --tracers 1 --rounds 15 --burst 80 \
      union= off=FESOM2_P1V_UNION=0 union_b= off_b=FESOM2_P1V_UNION=0 > gpurun_out/s18_ab_${mesh}_1.txt 2>&1
done
echo "ab done"
