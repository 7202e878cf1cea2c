#!/bin/bash
# Round 5: the LDS-stash p1v form at 64 VGPRs / 8 waves per SIMD (one 16-B LDS store per stashed
# level pair instead of two 8-B ones: 66 -> 64 VGPRs, no spills) against the previous build
# (fesom2-accelerate_amd/lib_r05base: a copy of lib/ built from the commit before, not kept in the tree;
# 66 VGPRs / 7 waves): parity first, then interleaved A/B of
# the single-tracer headline, 6 tracers and 9.6M x 80 on one GPU (the forms that take the stash).
set -eo pipefail
export TMPDIR=/tmp
export FESOM2_LIB_NAME=libfesom2-accelerate.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_batched.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "large_partition or plan_shapes or graph_after" > gpurun_out/r05e_stash8_tests.log 2>&1
echo "tests ok"
timeout -k 10 300 python bench.py --no-cpu-baseline --extras none > gpurun_out/r05e_stash8_1tr_check.json 2> gpurun_out/r05e_stash8_1tr_check.err
timeout -k 10 300 python bench.py --no-cpu-baseline --extras none --tracers 6 > gpurun_out/r05e_stash8_6tr_check.json 2> gpurun_out/r05e_stash8_6tr_check.err
echo "checks ok"
A="FESOM2_LIB_DIR=fesom2-accelerate_amd/lib_r05base"
B="FESOM2_LIB_DIR=fesom2-accelerate_amd/lib"
ROUNDS=4 STEPS=40 timeout -k 10 600 bash tools/sweep_env.sh "$A" "$B"
cp gpurun_out/sweep.txt gpurun_out/r05e_sweep_stash8_1tr.txt
ROUNDS=3 STEPS=20 BENCH_ARGS="--tracers 6" timeout -k 10 600 bash tools/sweep_env.sh "$A" "$B"
cp gpurun_out/sweep.txt gpurun_out/r05e_sweep_stash8_6tr.txt
echo "sweeps done"
