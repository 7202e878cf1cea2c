#!/usr/bin/env python3
"""Wave-state breakdown of the pass kernels from tools/sq_breakdown.sh's PMC passes.

SQ_WAVE_CYCLES splits (MI355X_MICROARCH.md, "rocprofv3 PMC slots") into SQ_WAIT_ANY (parked:
s_waitcnt or a barrier), SQ_WAIT_INST_ANY (ready but stalled at issue) and SQ_ACTIVE_INST_ANY
(issuing); the instruction counters give per-wave work.  Counts are averaged over the launches of a
kernel in the run and printed per launch.

usage: sq_breakdown.py DIR [OUT_JSON]   (DIR = gpurun_out/{sq,mem}_TAG, holding <workload>_{A,B,C}/ passes;
       tools/sq_breakdown.sh and tools/mem_breakdown.sh)
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import kernel_key  # noqa: E402


def per_kernel(path):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        acc[kernel_key(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def main():
    d = sys.argv[1]
    res = {}
    for csv_path in sorted(glob.glob(os.path.join(d, "*_[ABC]", "**", "*counter_collection.csv"), recursive=True)):
        wl = os.path.relpath(csv_path, d).split(os.sep)[0].rsplit("_", 1)[0]
        for k, cs in per_kernel(csv_path).items():
            res.setdefault(wl, {}).setdefault(k, {}).update(cs)
    out = {}
    for wl, ks in res.items():
        for k, c in sorted(ks.items()):
            wc = c.get("SQ_WAVE_CYCLES")
            waves = c.get("SQ_WAVES")
            row = {"counters": c}
            if wc:
                for name, key in (("parked", "SQ_WAIT_ANY"), ("issue_stall", "SQ_WAIT_INST_ANY"),
                                  ("issuing", "SQ_ACTIVE_INST_ANY"), ("valu", "SQ_ACTIVE_INST_VALU"),
                                  ("vmem", "SQ_ACTIVE_INST_VMEM"), ("lds", "SQ_ACTIVE_INST_LDS")):
                    if key in c:
                        row[name + "_frac"] = c[key] / wc
            if waves:
                for name, key in (("valu_per_wave", "SQ_INSTS_VALU"), ("vmem_rd_per_wave", "SQ_INSTS_VMEM_RD"),
                                  ("vmem_wr_per_wave", "SQ_INSTS_VMEM_WR"), ("lds_per_wave", "SQ_INSTS_LDS"),
                                  ("salu_per_wave", "SQ_INSTS_SALU"), ("wave_cycles_per_wave", "SQ_WAVE_CYCLES")):
                    if key in c:
                        row[name] = c[key] / waves
            def ratio(name, num, den, scale=1.0):
                if num in c and c.get(den):
                    row[name] = scale * c[num] / c[den]
            ratio("l2_read_latency_cycles", "TCP_TCC_READ_REQ_LATENCY_sum", "TCP_TCC_READ_REQ_sum")
            ratio("dram_read_queue_level", "TCC_EA0_RDREQ_LEVEL_sum", "TCC_EA0_RDREQ_sum")
            if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c and c["TCC_HIT_sum"] + c["TCC_MISS_sum"]:
                row["l2_hit_rate"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
            ratio("l1_accesses_per_l2_read", "TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum")
            if "SQ_LDS_BANK_CONFLICT" in c and "SQ_ACTIVE_INST_LDS" in c and c["SQ_ACTIVE_INST_LDS"]:
                row["lds_conflict_over_active"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_ACTIVE_INST_LDS"]
            out.setdefault(wl, {})[k] = row
            print(wl, k, " ".join(f"{n}={v:.3g}" for n, v in row.items() if n != "counters"))
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
