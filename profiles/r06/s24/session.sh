#!/bin/bash
# round 6 session 24: bench's batched legs with the same tracers timed as single-tracer passes in
# sequence (single_passes, batch_gain)
set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --no-cpu-baseline --legs config1_127kx47_6tracers,config3_1p2Mx80_6tracers \
    > gpurun_out/s24_bench.json 2> gpurun_out/s24_bench.err
echo "bench done"
