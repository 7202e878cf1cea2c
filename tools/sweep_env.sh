#!/bin/bash
# usage: tools/sweep_env.sh "ENV=.. ENV=.." "ENV=.." ...   (one bench run per argument)
set -o pipefail
out=gpurun_out/sweep.txt
: > $out
for cfg in "$@"; do
  env $cfg timeout -k 10 120 python bench.py --no-cpu-baseline --steps ${STEPS:-30} $BENCH_ARGS > gpurun_out/sw.json 2>gpurun_out/sw_err.log || exit 1
  python -c "
import json;d=json.load(open('gpurun_out/sw.json'))
k=d['kernels'];print('$cfg |', d['ms_per_step'], {n:v['avg_ms'] for n,v in k.items()})" >> $out
done
