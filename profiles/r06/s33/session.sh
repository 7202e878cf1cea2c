#!/bin/bash
# round 6 session 33: the product build's union plans at full size on unstructured numberings and
# meshes, each run checked cell for cell against the oracle
set -eo pipefail
export TMPDIR=/tmp
run() { name=$1; shift; timeout -k 10 400 python -u bench.py --extras none --no-cpu-baseline "$@" \
        > gpurun_out/s33_$name.json 2> gpurun_out/s33_$name.err; echo "$name done"; }
run dh127k6 --config '127k x 47' --tracers 6 --mesh delaunay-hilbert
run d127k1 --config '127k x 47' --mesh delaunay
run p127k6 --config '127k x 47' --tracers 6 --permuted
run dh127k1v --config '127k x 47' --mesh delaunay-hilbert --parity-levels
