#!/bin/bash
# round 6 session 2: the capped cluster-union p1v and tracer-group tile orders (tuning build):
# exactness, plan statistics, interleaved A/B at 127k x 47 (1 and 6 tracers) and 6 x 1.2M x 80
set -eo pipefail
export TMPDIR=/tmp
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_tuning.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "cluster_union or tracer_group" > gpurun_out/s2_tests.log 2>&1
echo "tests done"
st() {  # name env... -- bench args
  local n=$1; shift; local e=(); while [ "$1" != "--" ]; do e+=("$1"); shift; done; shift
  env "${e[@]}" FESOM2_PLAN_STATS=1 timeout -k 10 200 python bench.py --no-cpu-baseline --extras none --steps 3 --warmup 1 "$@" \
      > gpurun_out/s2_stats_$n.json 2> gpurun_out/s2_stats_$n.err
}
st u2 FESOM2_P1V_UNION=2 -- --config '127k x 47' --tracers 6
st u2rp FESOM2_P1V_UNION=2 FESOM2_ROWPAIR=1 -- --config '127k x 47' --tracers 6
st u2g16 FESOM2_P1V_UNION=2 FESOM2_ROWPAIR=1 FESOM2_GROUP=16 -- --config '127k x 47' --tracers 6
st u2big FESOM2_P1V_UNION=2 FESOM2_P1V_UNION_MAX=18 -- --tracers 6
echo "stats done"
SWEEP_OUT=gpurun_out/s2_sweep_127k6.txt ROUNDS=3 STEPS=80 BENCH_ARGS="--config '127k x 47' --tracers 6" timeout -k 10 600 \
    bash tools/sweep_env.sh "FESOM2_P1V_UNION=0" "FESOM2_P1V_UNION=2" "FESOM2_P1V_UNION=2 FESOM2_ROWPAIR=1" \
    "FESOM2_P1V_UNION=2 FESOM2_ROWPAIR=1 FESOM2_P1V_UNION_MAX=20" "FESOM2_P1V_UNION=2 FESOM2_ROWPAIR=1 FESOM2_GROUP=16" \
    "FESOM2_P1V_UNION=2 FESOM2_ROWPAIR=1 FESOM2_GROUP=16 FESOM2_P1V_UNION_MAX=36" "FESOM2_ROWPAIR=1" \
    "FESOM2_TRACER_GROUP=2" "FESOM2_TRACER_GROUP=3" "FESOM2_P1V_UNION=2 FESOM2_TRACER_GROUP=3"
echo "sweep 127k6 done"
SWEEP_OUT=gpurun_out/s2_sweep_127k1.txt ROUNDS=3 STEPS=400 BENCH_ARGS="--config '127k x 47'" timeout -k 10 400 \
    bash tools/sweep_env.sh "FESOM2_P1V_UNION=0" "FESOM2_P1V_UNION=2" "FESOM2_P1V_UNION=2 FESOM2_ROWPAIR=1" \
    "FESOM2_P1V_UNION=2 FESOM2_ROWPAIR=1 FESOM2_P1V_UNION_MAX=20" "FESOM2_P1V_UNION=2 FESOM2_ROWPAIR=1 FESOM2_GROUP=16"
echo "sweep 127k1 done"
SWEEP_OUT=gpurun_out/s2_sweep_1p2M6.txt ROUNDS=2 STEPS=10 BENCH_ARGS="--tracers 6" timeout -k 10 400 \
    bash tools/sweep_env.sh "FESOM2_P1V_UNION=0" "FESOM2_P1V_UNION=2 FESOM2_P1V_UNION_MAX=18" \
    "FESOM2_P1V_UNION=2 FESOM2_P1V_UNION_MAX=18 FESOM2_P1V_STASH=0"
echo "sweep 1p2M6 done"
