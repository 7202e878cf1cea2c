#!/bin/bash
# A/B sweep of environment knobs: tools/sweep_env.sh "ENV=.. ENV=.." "ENV=.." ...
# Runs every configuration ROUNDS times, interleaved (A B C A B C ...), because the GPU's clocks
# drift over minutes of back-to-back runs; one line per run in gpurun_out/sweep.txt.
# A configuration may carry bench arguments after " | " ("FESOM2_X=1 | --path split").
# BENCH_ARGS (eval'ed: may quote), STEPS, ROUNDS, SWEEP_OUT (default gpurun_out/sweep.txt).
set -o pipefail
# the knobs exist in the tuning build only (make -C fesom2-accelerate_amd tuning)
export FESOM2_LIB_NAME=${FESOM2_LIB_NAME:-libfesom2-accelerate-tuning.so}
out=${SWEEP_OUT:-gpurun_out/sweep.txt}
: > $out
for r in $(seq 1 ${ROUNDS:-1}); do
  for cfg in "$@"; do
    envs=${cfg%%|*}
    args=""
    [[ "$cfg" == *"|"* ]] && args=${cfg#*|}
    eval "env $envs timeout -k 10 120 python bench.py --no-cpu-baseline --no-check --extras none --steps ${STEPS:-30} $BENCH_ARGS $args" \
        > gpurun_out/sw.json 2> gpurun_out/sw_err.log || exit 1
    python -c "
import json;d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1])
k=d['kernels'];print('r$r $cfg |', d['ms_per_step'], {n:v['avg_ms'] for n,v in k.items()})" >> $out
  done
done
