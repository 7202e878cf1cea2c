#!/bin/bash
# Where the batched p1v's extra L2-miss traffic comes from (BASELINE config 3, 6 x 1.2M x 80), on the
# tuning build: for each variant one timing run of bench.py (the kernels' own HIP events) and one
# rocprofv3 PMC pass of the L2 -> fabric read requests (profiles/pmc_traffic.py turns them into
# bytes).  Variants: the default plan; no cluster gathers / no edge gathers (FESOM2_ABLATE 1 / 2,
# timing only: results wrong); single rows without the stash; row pairs in 1024-node patches;
# strips of 18 / 24 nodes inside the patches (FESOM2_BATCH_STRIP, strip_order).
# usage (on the GPU box): [ABL_ARGS="--config '127k x 47' --tracers 6"] bash tools/pmc_batch_ablate.sh TAG [variant ...]
#   (ABL_ARGS: the workload, default --tracers 6)
set -eo pipefail
tag=${1:-r05}
shift || true
export TMPDIR=/tmp
export FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so
declare -A V=(
  [default]=""
  [nocluster]="FESOM2_ABLATE=1"
  [noedge]="FESOM2_ABLATE=2"
  [singlerow]="FESOM2_ROWPAIR=0 FESOM2_P1V_STASH=0"
  [patch1024]="FESOM2_BATCH_PATCH=1024"
  [strip18]="FESOM2_BATCH_STRIP=18"
  [strip24]="FESOM2_BATCH_STRIP=24"
)
names=("$@")
[ ${#names[@]} -eq 0 ] && names=(default nocluster noedge singlerow patch1024)
eval "wl=(${ABL_ARGS:---tracers 6})"
args=("${wl[@]}" --no-cpu-baseline --no-check --extras none)
for v in "${names[@]}"; do
  out=gpurun_out/pmcab_${tag}_$v
  rm -rf "$out" && mkdir -p "$out"
  env ${V[$v]} timeout -k 10 240 python3 bench.py "${args[@]}" --kernel-timing all --steps 10 --warmup 2 \
      > "$out/bench.json" 2> "$out/bench.err"
  env ${V[$v]} timeout -k 10 240 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum \
      --output-format csv -d "$out/rd" -o rd -- python3 bench.py "${args[@]}" --steps 3 --warmup 1 \
      > /dev/null 2> "$out/rd.err"
  echo "variant $v done"
done
