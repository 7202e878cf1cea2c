#!/bin/bash
# round 6 session 25: the default bench after the single_passes comparator (every leg)
set -eo pipefail
export TMPDIR=/tmp
start=$(date +%s)
timeout -k 10 900 python -u bench.py > gpurun_out/s25_bench.json 2> gpurun_out/s25_bench.err
echo "bench done in $(( $(date +%s) - start )) s"
