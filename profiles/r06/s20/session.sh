#!/bin/bash
# round 6 session 20: the partitioned split pass with cluster unions (new tests), then the round-end
# rehearsal: GPU suite, smoke, default bench
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k split_pass_with --timeout 120 \
    --timeout-method thread > gpurun_out/s20_newtests.log 2>&1
rc=$?
echo "new tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q --timeout 600 --timeout-method thread \
    > gpurun_out/s20_gputests.log 2>&1
rc=$?
echo "gpu tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s20_smoke.log 2>&1 || exit $?
echo "smoke done"
timeout -k 10 900 python -u bench.py > gpurun_out/s20_bench.json 2> gpurun_out/s20_bench.err || exit $?
echo "bench done"
