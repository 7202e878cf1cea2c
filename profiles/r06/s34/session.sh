#!/bin/bash
# round 6 session 34: the N > 1 bench path (2 and 3 ranks on one GPU, host exchange) as -m gpu tests
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py -m gpu -v --timeout 600 --timeout-method thread \
    > gpurun_out/s34_tests.log 2>&1
echo "rc=$?"
