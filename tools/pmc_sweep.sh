#!/bin/bash
# Read traffic (L2 -> fabric requests, PMC) of each kernel under environment variants:
#   tools/pmc_sweep.sh "ENV=.." "ENV=.." ...     (one rocprofv3 --pmc pass per configuration)
# One line per configuration in gpurun_out/pmc_sweep.txt: kernel -> read GB, and the bench's ms/pass.
set -eo pipefail
export TMPDIR=/tmp
out=gpurun_out/pmc_sweep.txt
: > $out
i=0
for cfg in "$@"; do
  i=$((i+1))
  d=gpurun_out/pmcs_$i
  rm -rf $d && mkdir -p $d
  eval "env $cfg timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum \
      --output-format csv -d $d/rd -o rd -- python3 bench.py --no-cpu-baseline --no-check --extras none --steps 3 --warmup 1 $BENCH_ARGS" \
      > $d/bench.json 2> $d/err.log
  python3 - "$cfg" $d >> $out <<'PY'
import csv, collections, glob, json, sys
cfg, d = sys.argv[1], sys.argv[2]
sys.path.insert(0, "profiles")
from pmc_traffic import kernel_key
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + "/rd/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[kernel_key(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {}
for k, cs in acc.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    res[k] = round((128 * m.get("TCC_EA0_RDREQ_128B_sum", 0) + 64 * m.get("TCC_EA0_RDREQ_64B_sum", 0)
                    + 32 * m.get("TCC_EA0_RDREQ_32B_sum", 0)) / 1e9, 3)
b = json.loads(open(d + "/bench.json").read().strip().splitlines()[-1])
print(cfg, "| read GB", res, "| ms", b["ms_per_step"], {n: v["avg_ms"] for n, v in b["kernels"].items()})
PY
done
