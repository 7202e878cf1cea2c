#!/bin/bash
# round 6: rocprofv3 kernel-trace stats + PMC traffic of the final product build for every workload
# the bench reports traffic for; each traffic file is stamped on the box with the code-object hash
# of the library that ran (tools/profile.sh TRAFFIC_OUT -> profiles/pmc_traffic.py)
set -eo pipefail
export TMPDIR=/tmp
p() {  # tag out workload tracers [emulate] -- bench args (BENCH_ARGS string)
  TRAFFIC_OUT=$2 TRAFFIC_WL="$3" TRAFFIC_TR=$4 TRAFFIC_EMU="$5" TRAFFIC_SRC="round 6 final build: profiles/r06/prof_$1" \
      timeout -k 10 900 bash tools/profile.sh "$1"
  echo "profile $1 done"
}
BENCH_ARGS="" p r06_1p2M traffic.json "1.2M x 80" 1
BENCH_ARGS="--config '127k x 47'" p r06_127k traffic_127kx47.json "127k x 47" 1
BENCH_ARGS="--config '127k x 47' --tracers 6" p r06_127k6 traffic_127kx47_6tr.json "127k x 47" 6
BENCH_ARGS="--tracers 6" p r06_1p2M6 traffic_1p2Mx80_6tr.json "1.2M x 80" 6
BENCH_ARGS="--scaling strong --emulate-rank 3/8" p r06_rank3of8 traffic_9p6Mx80_rank3of8.json "9.6M x 80" 1 3/8
BENCH_ARGS="--scaling strong" p r06_9p6M traffic_9p6Mx80.json "9.6M x 80" 1
# the union plans' effect on the memory pipeline (127k x 47, 6 tracers: product default against
# FESOM2_P1V_UNION=0), and the unions forced onto the large partition (6 x 1.2M x 80)
timeout -k 10 900 bash tools/mem_breakdown.sh r06u "u127k6|--config '127k x 47' --tracers 6" \
    "off127k6|--config '127k x 47' --tracers 6|FESOM2_P1V_UNION=0" "u1p2M6|--tracers 6|FESOM2_P1V_UNION=1" \
    "d1p2M6|--tracers 6"
echo "mem breakdown done"
