#!/bin/bash
# round 6 session 23 (product build): six tracers as single-tracer passes on 1/2/3/6 streams against
# the batched entries
set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/streams_ab.py --config '127k x 47' --tracers 6 --streams 1,2,3,6 --rounds 15 \
    --burst 20 > gpurun_out/s23_streams_127k6.txt 2>&1
echo "127k done"
timeout -k 10 500 python -u tools/streams_ab.py --config '1.2M x 80' --tracers 6 --streams 1,2,3 --rounds 7 \
    --burst 4 > gpurun_out/s23_streams_1p2M6.txt 2>&1
echo "1.2M done"
