#!/bin/bash
# PMC read/write traffic of the default bench under FESOM2_ABLATE variants (timing-only builds)
set -eo pipefail
export TMPDIR=/tmp
for ab in 0 1 2 3; do
  out=gpurun_out/pmc_ab$ab
  rm -rf "$out" && mkdir -p "$out"
  FESOM2_ABLATE=$ab timeout -k 10 200 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum \
      --output-format csv -d "$out/rd" -o rd -- python3 bench.py --no-cpu-baseline --no-check --extras none --steps 2 --warmup 1 > /dev/null 2> "$out/rd.err"
  FESOM2_ABLATE=$ab timeout -k 10 200 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
      --output-format csv -d "$out/wr" -o wr -- python3 bench.py --no-cpu-baseline --no-check --extras none --steps 2 --warmup 1 > /dev/null 2> "$out/wr.err"
done
