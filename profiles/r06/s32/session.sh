#!/bin/bash
# round 6 session 32: final rehearsal of the round-end runs on the final tree -- GPU suite, smoke,
# default bench (product code object e31318456383f202)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q --timeout 600 --timeout-method thread \
    > gpurun_out/s32_gputests.log 2>&1
rc=$?
echo "gpu tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s32_smoke.log 2>&1 || exit $?
echo "smoke done"
timeout -k 10 900 python -u bench.py > gpurun_out/s32_bench.json 2> gpurun_out/s32_bench.err || exit $?
echo "bench done"
