#!/bin/bash
# round 6 session 13: after the mesh-info extension -- GPU suite, smoke, default bench
set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 600 --timeout-method thread \
    > gpurun_out/s13_gputests.log 2>&1
echo "gpu tests done"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s13_smoke.log 2>&1
echo "smoke done"
timeout -k 10 900 python -u bench.py > gpurun_out/s13_bench.json 2> gpurun_out/s13_bench.err
echo "bench done"
