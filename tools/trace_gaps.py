#!/usr/bin/env python3
"""Per-launch durations and the idle gaps between consecutive kernels from a rocprofv3 kernel trace.

usage: tools/trace_gaps.py <dir with *kernel_trace.csv> [--last N]

For every pass (p1v -> b3h -> p2h) of the timed region it reports each kernel's duration and the
gap from the previous kernel's end to its start -- the launch/ramp overhead that a small partition
(127k x 47: 0.3 ms per pass) pays three times per pass.  Only the last N launches of each kernel
are used (the timed steps; the warmup and the check pass come earlier or later and are dropped by
--skip-tail).
"""
import argparse
import csv
import glob
import os
import statistics


def short(name):
    for k, s in (("k_p1", "p1v"), ("k_b3h", "b3h"), ("k_p2h", "p2h"), ("k_p2", "p2"), ("k_b3v", "b3v"), ("k_c", "c")):
        if k in name:
            return s
    return name.split("(")[0][-24:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=60, help="launches of the trace's end to use")
    ap.add_argument("--skip-tail", type=int, default=0, help="drop this many launches at the very end")
    args = ap.parse_args()
    files = glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel_trace.csv under {args.dir}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    if args.skip_tail:
        rows = rows[: -args.skip_tail]
    rows = rows[-args.last:]
    dur, gap = {}, {}
    for i, (s, e, k) in enumerate(rows):
        dur.setdefault(k, []).append((e - s) / 1e3)
        if i:
            gap.setdefault(k, []).append((s - rows[i - 1][1]) / 1e3)
    span = (rows[-1][1] - rows[0][0]) / 1e3
    busy = sum(e - s for s, e, _ in rows) / 1e3
    print(f"{len(rows)} launches over {span:.1f} us, kernels busy {busy:.1f} us ({100 * busy / span:.1f} %)")
    for k in dur:
        d, g = dur[k], gap.get(k, [0.0])
        print(f"  {k:6s} n={len(d):3d} dur median {statistics.median(d):8.2f} us   gap before median "
              f"{statistics.median(g):6.2f} us (min {min(g):6.2f}, max {max(g):7.2f})")


if __name__ == "__main__":
    main()
