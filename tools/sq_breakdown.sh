#!/bin/bash
# SQ (wave-state) breakdown of the pass kernels: where p1v's wave cycles go -- parked on memory
# (SQ_WAIT_ANY), stalled at issue (SQ_WAIT_INST_ANY) or issuing (SQ_ACTIVE_INST_*) -- single tracer
# against the 6-tracer batch.  Two PMC passes per workload, 8 SQ counters each, no tracing combined;
# counters the box does not list are dropped (rocprofv3 -L) so a pass never asks for an unknown name.
# usage (on the GPU box): bash tools/sq_breakdown.sh TAG   -> gpurun_out/sq_TAG/{list.txt,<wl>_<pass>/...}
set -eo pipefail
tag=${1:-r05}
export TMPDIR=/tmp
out=gpurun_out/sq_$tag
rm -rf "$out" && mkdir -p "$out"
timeout -k 10 120 rocprofv3 -L > "$out/list.txt" 2> "$out/list.err"
have() { for c in "$@"; do grep -qw "$c" "$out/list.txt" && printf '%s ' "$c"; done; }
A=$(have SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM)
B=$(have SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS)
echo "pass A: $A" > "$out/passes.txt"
echo "pass B: $B" >> "$out/passes.txt"
run() {  # workload-name pass-name counters... -- bench args...
    local wl=$1 ps=$2; shift 2
    local ctr=()
    while [ "$1" != "--" ]; do ctr+=("$1"); shift; done
    shift
    timeout -k 10 -s KILL 180 rocprofv3 --pmc "${ctr[@]}" --output-format csv -d "$out/${wl}_$ps" -o pmc -- \
        python3 bench.py --no-cpu-baseline --no-check --extras none --steps 3 --warmup 1 "$@" \
        > "$out/${wl}_$ps.json" 2> "$out/${wl}_$ps.err"
}
run 1p2M A $A --
run 1p2M B $B --
run 6tr A $A -- --tracers 6
run 6tr B $B -- --tracers 6
run 127k6 A $A -- --tracers 6 --config "127k x 47"
run 127k6 B $B -- --tracers 6 --config "127k x 47"
find "$out" -name "*.csv" | sort > "$out/files.txt"
echo "sq breakdown done"
