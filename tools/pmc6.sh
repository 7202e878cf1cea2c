#!/bin/bash
# PMC traffic of the 6-tracer batched pass (same counters as tools/profile.sh)
set -eo pipefail
export TMPDIR=/tmp
out=gpurun_out/prof_6tr
rm -rf "$out" && mkdir -p "$out"
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum \
    --output-format csv -d "$out/rd" -o rd -- python3 bench.py --tracers 6 --no-cpu-baseline --no-check --extras none --steps 3 --warmup 1 \
    > /dev/null 2> "$out/rd.err"
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
    --output-format csv -d "$out/wr" -o wr -- python3 bench.py --tracers 6 --no-cpu-baseline --no-check --extras none --steps 3 --warmup 1 \
    > /dev/null 2> "$out/wr.err"
