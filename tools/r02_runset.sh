set -e
run() { name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/r02c_$name.json 2> gpurun_out/r02c_$name.err; tail -1 gpurun_out/r02c_$name.json | cut -c1-120; }
run default
run vlimit2_check --vlimit 2 --check --no-cpu-baseline
run vlimit3_check --vlimit 3 --check --no-cpu-baseline
run iter2_check --fct-iter 2 --check --no-cpu-baseline --steps 10
run fused_check --path fused --check --no-cpu-baseline
run reference_check --path reference --check --no-cpu-baseline
run graph_check --graph --check --no-cpu-baseline
run strong_9p6M --scaling strong --no-cpu-baseline --steps 10 --warmup 3
