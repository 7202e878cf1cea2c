#!/bin/bash
# Memory-pipeline counters of the pass kernels (where p1v's requests queue): average L2 read latency
# seen by the L1 (TCP_TCC_READ_REQ_LATENCY / TCP_TCC_READ_REQ), L2 hit rate, DRAM read queue level
# (TCC_EA0_RDREQ_LEVEL / TCC_EA0_RDREQ), TA/TD busy and stall cycles -- single tracer against the
# 6-tracer batch.  Three PMC passes per workload within the per-block limits (<= 4 TCP, 4 TCC, 2 TA,
# 2 TD, 2 GRBM), no tracing combined; names the box does not list are dropped (rocprofv3 -L).
# usage (on the GPU box): bash tools/mem_breakdown.sh TAG ['name|bench args' ...]  -> gpurun_out/mem_TAG/...
#   default workloads: 1p2M (the headline) and 6tr (--tracers 6); e.g. the 127k x 47 pair:
#   bash tools/mem_breakdown.sh r06 "127k|--config '127k x 47'" "127k6|--config '127k x 47' --tracers 6"
#   (a third field sets environment variables for that workload: "off|--tracers 6|FESOM2_P1V_UNION=0")
set -eo pipefail
tag=${1:-r05}
shift || true
wls=("$@")
[ ${#wls[@]} -eq 0 ] && wls=("1p2M|" "6tr|--tracers 6")
export TMPDIR=/tmp
out=gpurun_out/mem_$tag
rm -rf "$out" && mkdir -p "$out"
timeout -k 10 120 rocprofv3 -L > "$out/list.txt" 2> "$out/list.err"
have() { for c in "$@"; do grep -qw "$c" "$out/list.txt" && printf '%s ' "$c"; done; }
A=$(have TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT)
B=$(have TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_TAG_STALL_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum TD_TD_BUSY_sum TD_TC_STALL_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_TOTAL_WAVEFRONTS_sum)
C=$(have TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_BUSY_sum)
{ echo "pass A: $A"; echo "pass B: $B"; echo "pass C: $C"; } > "$out/passes.txt"
run() {  # workload pass counters... -- bench args...   (WL_ENV: K=V ... for this workload)
    local wl=$1 ps=$2; shift 2
    local ctr=()
    while [ "$1" != "--" ]; do ctr+=("$1"); shift; done
    shift
    env ${WL_ENV:-} timeout -k 10 -s KILL 180 rocprofv3 --pmc "${ctr[@]}" --output-format csv -d "$out/${wl}_$ps" -o pmc -- \
        python3 bench.py --no-cpu-baseline --no-check --extras none --steps 3 --warmup 1 "$@" \
        > "$out/${wl}_$ps.json" 2> "$out/${wl}_$ps.err"
}
for ps in A B C; do
    eval "ctr=\$$ps"
    for w in "${wls[@]}"; do
        rest=${w#*|}
        WL_ENV=""
        if [[ "$rest" == *"|"* ]]; then WL_ENV=${rest#*|}; rest=${rest%%|*}; fi  # name|args|K=V K=V
        eval "wargs=($rest)"
        WL_ENV="$WL_ENV" run "${w%%|*}" $ps $ctr -- "${wargs[@]}"
    done
done
find "$out" -name "*.csv" | sort > "$out/files.txt"
echo "mem breakdown done"
