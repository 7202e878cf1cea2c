#!/bin/bash
# rocprofv3 evidence for profiles/: kernel-trace stats of the default bench command, then the two
# PMC passes (L2->fabric read / write requests; separate runs, no tracing combined with --pmc).
# usage (on the GPU box): [BENCH_ARGS="--config '127k x 47'"] bash tools/profile.sh TAG
# With TRAFFIC_OUT=profiles/traffic_X.json TRAFFIC_WL="127k x 47" [TRAFFIC_TR=6] [TRAFFIC_EMU=3/8] the
# PMC passes become that traffic file on the box itself, stamped with the code-object hash of the
# library that ran them (profiles/pmc_traffic.py; copy it back from gpurun_out/prof_TAG/).
set -eo pipefail
tag=${1:-r01}
export TMPDIR=/tmp
eval "args=(${BENCH_ARGS:-})"
out=gpurun_out/prof_$tag
rm -rf "$out" && mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d "$out/stats" -o run -- \
    python3 bench.py --no-cpu-baseline --no-check --extras none "${args[@]}" > "$out/bench_under_rocprof.json" 2> "$out/stats.err"
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum \
    --output-format csv -d "$out/rd" -o rd -- python3 bench.py --no-cpu-baseline --no-check --extras none --steps 3 --warmup 1 "${args[@]}" \
    > /dev/null 2> "$out/rd.err"
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
    --output-format csv -d "$out/wr" -o wr -- python3 bench.py --no-cpu-baseline --no-check --extras none --steps 3 --warmup 1 "${args[@]}" \
    > /dev/null 2> "$out/wr.err"
find "$out" -name "*.csv" | sort > "$out/files.txt"
if [ -n "${TRAFFIC_OUT:-}" ]; then
    emu=()
    [ -n "${TRAFFIC_EMU:-}" ] && emu=(--emulate "$TRAFFIC_EMU")
    python3 profiles/pmc_traffic.py "$(find "$out/rd" -name '*counter_collection.csv' | head -1)" \
        "$(find "$out/wr" -name '*counter_collection.csv' | head -1)" "$TRAFFIC_WL" "$out/$(basename "$TRAFFIC_OUT")" \
        "${TRAFFIC_TR:-1}" "${TRAFFIC_SRC:-$tag}" "${emu[@]}" > /dev/null
fi
