#!/bin/bash
# round 6 session 21: the partitioned split-pass tests with cluster unions (fixed), the partitioned
# fused-pass tests beside them
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "split_pass_with or partitioned_pass" \
    --timeout 120 --timeout-method thread > gpurun_out/s21_tests.log 2>&1
echo "rc=$?"
