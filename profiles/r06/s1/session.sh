#!/bin/bash
# round 6 session 1: (a) why batching does not pay at 127k x 47 -- memory-pipeline
# counters and per-kernel L2->fabric reads, 1 tracer against the 6-tracer batch, with the cluster/edge
# gather ablations; (b) the cluster-union p1v: exactness on the tuning build, its
# plan statistics, and an interleaved A/B at 127k x 47 (1 and 6 tracers) and 1.2M x 80 (1 and 6)
set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 400 bash tools/mem_breakdown.sh r06a "127k|--config '127k x 47'" "127k6|--config '127k x 47' --tracers 6"
echo "mem done"
ABL_ARGS="--config '127k x 47' --tracers 6" timeout -k 10 300 bash tools/pmc_batch_ablate.sh r06a_127k6 default nocluster noedge
echo "abl6 done"
ABL_ARGS="--config '127k x 47'" timeout -k 10 300 bash tools/pmc_batch_ablate.sh r06a_127k1 default nocluster noedge
echo "abl1 done"
FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so timeout -k 10 300 python -u -m pytest tests/test_gpu_tuning.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -k cluster_union > gpurun_out/s1_union_tests.log 2>&1
echo "union tests done"
for c in "1p2M|" "1p2M6|--tracers 6" "127k|--config '127k x 47'" "127k6|--config '127k x 47' --tracers 6"; do
  eval "a=(${c#*|})"
  FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so FESOM2_PLAN_STATS=1 FESOM2_P1V_UNION=1 timeout -k 10 200 \
      python bench.py --no-cpu-baseline --extras none --steps 5 --warmup 1 "${a[@]}" > gpurun_out/s1_union_${c%%|*}.json 2> gpurun_out/s1_union_${c%%|*}.err
done
echo "union checks done"
SWEEP_OUT=gpurun_out/s1_sweep_127k6.txt ROUNDS=3 STEPS=80 BENCH_ARGS="--config '127k x 47' --tracers 6" timeout -k 10 300 \
    bash tools/sweep_env.sh "FESOM2_P1V_UNION=0" "FESOM2_P1V_UNION=1" "FESOM2_P1V_UNION=2"
SWEEP_OUT=gpurun_out/s1_sweep_127k1.txt ROUNDS=3 STEPS=400 BENCH_ARGS="--config '127k x 47'" timeout -k 10 300 \
    bash tools/sweep_env.sh "FESOM2_P1V_UNION=0" "FESOM2_P1V_UNION=1" "FESOM2_P1V_UNION=2"
SWEEP_OUT=gpurun_out/s1_sweep_1p2M6.txt ROUNDS=3 STEPS=10 BENCH_ARGS="--tracers 6" timeout -k 10 400 \
    bash tools/sweep_env.sh "FESOM2_P1V_UNION=0" "FESOM2_P1V_UNION=1" "FESOM2_P1V_UNION=2"
SWEEP_OUT=gpurun_out/s1_sweep_1p2M1.txt ROUNDS=3 STEPS=30 timeout -k 10 300 \
    bash tools/sweep_env.sh "FESOM2_P1V_UNION=0" "FESOM2_P1V_UNION=1" "FESOM2_P1V_UNION=2"
echo "sweeps done"
