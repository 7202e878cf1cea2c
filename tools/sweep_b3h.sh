#!/bin/bash
# b3h variants: U (groups per block) x NT
set -o pipefail
for cfg in "1 0" "2 0" "4 0" "8 0" "1 1" "2 1" "4 1"; do
  set -- $cfg
  FESOM2_B3H_U=$1 FESOM2_B3H_NT=$2 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/sw_$1_$2.json 2>gpurun_out/sw_err.log || exit 1
  python -c "
import json;d=json.load(open('gpurun_out/sw_$1_$2.json'))
k=d['kernels'];print('U=$1 NT=$2', d['ms_per_step'], {n:v['avg_ms'] for n,v in k.items()})" >> gpurun_out/sweep.txt
done
