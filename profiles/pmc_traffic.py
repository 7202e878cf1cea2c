#!/usr/bin/env python3
"""Turn rocprofv3 PMC passes into HBM bytes per kernel launch (profiles/traffic.json).

Method (MI355X_MICROARCH.md "HBM", calibrated in this repo): FETCH_SIZE reads half of the bytes of
a coalesced stream on gfx950, so the L2->fabric request counters are used instead.  Calibration on
the stepwise k_a1 kernel, which reads exactly 2 x 768 MB and writes 2 x 768 MB at 1.2M x 80
(profiles/r01_calibration_stepwise_*.csv): TCC_EA0_RDREQ_128B_sum = 12.0e6 (x 128 B = 1.536 GB) and
TCC_EA0_WRREQ_64B_sum = 24.0e6 (x 64 B = 1.536 GB).  So

    read bytes  = 128 * RDREQ_128B + 64 * RDREQ_64B + 32 * RDREQ_32B
    write bytes = 64 * WRREQ_64B + 32 * (WRREQ - WRREQ_64B)

(the counters include Infinity-Cache hits: this is L2-miss traffic, an upper bound on HBM bytes).

Each file is stamped with the code-object hash of the engine library the PMC passes ran
(``code_object``: sha256 of its .hip_fatbin section, fesom2_amd._paths.code_object_hash) and the
kernel symbols rocprofv3 reported; bench.py reports the traffic only for a library with the same
kernels (``traffic_stale`` otherwise).

usage: pmc_traffic.py READ_CSV WRITE_CSV WORKLOAD OUT_JSON [TRACERS [SOURCE]] [--lib SO] [--emulate R/N]
"""
import collections
import argparse
import csv
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fesom2-accelerate_amd"))

NAMES = {"k_p1": "fct_ale_p1", "k_p1v": "fct_ale_p1v", "k_p2": "fct_ale_p2", "k_p2h": "fct_ale_p2h",
         "k_b3h_g": "fct_ale_b3_horizontal", "k_b3h_u": "fct_ale_b3_horizontal",
         "k_b3h_p": "fct_ale_b3_horizontal", "k_p2f": "fct_ale_p2_b3h"}


def kernel_key(name):
    """rocprof kernel name -> short name; k_p1<..., VERT = true> is the phase-1 + vertical kernel."""
    base = name.split("(")[0].replace("void ", "").replace("f2a::", "").strip()
    k = base.split("<")[0]
    args = [x.strip() for x in base[len(k) + 1:].rstrip(">").split(",")] if "<" in base else []
    if k == "k_p1" and len(args) > 5 and args[5] == "true":  # k_p1<VLIMIT, C, RB, EB, NT, VERT, OPT>
        return "k_p1v"
    return k


def per_kernel(path, symbols=None):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        k = kernel_key(r["Kernel_Name"])
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if symbols is not None:
            symbols.setdefault(k, set()).add(r["Kernel_Name"].split("(")[0].replace("void ", "").strip())
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("rd")
    ap.add_argument("wr")
    ap.add_argument("workload")
    ap.add_argument("out")
    ap.add_argument("tracers", nargs="?", type=int, default=1)
    ap.add_argument("source", nargs="?", default="")
    ap.add_argument("--lib", default=None, help="the engine library the passes ran (default: the product build)")
    ap.add_argument("--emulate", default=None, help="R/N: bench.py --emulate-rank R/N (one rank's strip)")
    a = ap.parse_args()
    rd, wr, workload, out, tracers, source = a.rd, a.wr, a.workload, a.out, a.tracers, a.source
    from fesom2_amd import _paths
    code = _paths.code_object_hash(a.lib)
    symbols = {}
    R, W = per_kernel(rd, symbols), per_kernel(wr, symbols)
    res = {}
    for k, name in NAMES.items():
        if k not in R or k not in W:
            continue
        r, w = R[k], W[k]
        rb = 128 * r.get("TCC_EA0_RDREQ_128B_sum", 0) + 64 * r.get("TCC_EA0_RDREQ_64B_sum", 0) + \
            32 * r.get("TCC_EA0_RDREQ_32B_sum", 0)
        wb = 64 * w.get("TCC_EA0_WRREQ_64B_sum", 0) + 32 * (w.get("TCC_EA0_WRREQ_sum", 0) -
                                                            w.get("TCC_EA0_WRREQ_64B_sum", 0))
        res[name] = {"read_bytes": int(rb), "write_bytes": int(wb), "total": int(rb + wb),
                     "symbol": sorted(symbols.get(k, ()))}
    doc = {"workload": workload, "tracers": tracers, "bytes_per_launch": {k: v["total"] for k, v in res.items()},
           "detail": res, "method": __doc__.strip().splitlines()[0] + " -- see profiles/pmc_traffic.py",
           "source": source, "code_object": code}
    if a.emulate:
        doc["emulate"] = a.emulate
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
