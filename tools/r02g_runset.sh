#!/bin/bash
# Final round-2 bench lines (r02g: + regular b3h packing) (run on the GPU box from the repo root): every --check run compares every
# owned cell with the oracle.  Output: gpurun_out/r02g_<name>.json (+ .err)
set -e
run() { name=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/r02g_$name.json 2> gpurun_out/r02g_$name.err; tail -1 gpurun_out/r02g_$name.json | cut -c1-150; }
run default
run 127k47_check --config "127k x 47" --check --no-cpu-baseline
run 6tracers_check --tracers 6 --check --no-cpu-baseline
run parity_levels_check --parity-levels --check --no-cpu-baseline
run graph_check --graph --check --no-cpu-baseline
run reference_check --path reference --check --no-cpu-baseline
run delaunay_check --mesh delaunay --check --no-cpu-baseline
run strong_9p6M --scaling strong --no-cpu-baseline --steps 10 --warmup 3
run delaunay_hilbert_check --mesh delaunay-hilbert --check --no-cpu-baseline
run vlimit2_check --vlimit 2 --check --no-cpu-baseline
run iter2_check --fct-iter 2 --check --no-cpu-baseline --steps 10
