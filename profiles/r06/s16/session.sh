#!/bin/bash
# round 6 session 16: the whole tuning-build suite (its launch-time knobs now take effect per test)
# and the product's plan-option tests with the cluster-union options
set -eo pipefail
export TMPDIR=/tmp
FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so timeout -k 10 900 python -u -m pytest tests/test_gpu_tuning.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/s16_tuning_tests.log 2>&1
echo "tuning suite done"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "plan_options or level_counts or degenerate" > gpurun_out/s16_parity_tests.log 2>&1
echo "parity subset done"
