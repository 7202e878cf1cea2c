#!/usr/bin/env python3
"""In-process interleaved A/B of tuning-build variants: one mesh, one set of field buffers, one set
of mesh handles and plans per variant, the variants' passes alternating in short bursts inside ONE
process, so clock and thermal drift (which moves separate bench.py runs by up to 7 % on some boxes)
hits every variant alike.

Each variant is a set of FESOM2_* knobs (tuning build, FESOM2_LIB_NAME): they are set while the
variant's plans are built (fesom2_prepare_mesh_) and again around each of its bursts (the launch-time
knobs).  Timing: a burst of K direction-split passes bracketed by device syncs; per variant the median
burst over R rounds, in ms per pass, plus the kernels' event timings over one extra burst.

usage: FESOM2_LIB_NAME=libfesom2-accelerate-tuning.so python tools/ab_inproc.py
           [--config '127k x 47'] [--tracers 6] [--rounds 15] [--burst 20] NAME=K1=V1,K2=V2 ...
       (a variant with no knobs: NAME=)
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fesom2-accelerate_amd"))

from fesom2_amd import abi, engine, synth  # noqa: E402


def parse_variant(s):
    name, _, knobs = s.partition("=")
    env = dict(kv.split("=", 1) for kv in knobs.split(",") if kv)
    return name, env


class Knobs:
    """Set a variant's knobs for a with-block (every knob any variant uses is reset first)."""

    def __init__(self, env, all_keys):
        self.env, self.keys = env, all_keys

    def __enter__(self):
        for k in self.keys:
            os.environ.pop(k, None)
        os.environ.update(self.env)

    def __exit__(self, *a):
        for k in self.keys:
            os.environ.pop(k, None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="127k x 47")
    ap.add_argument("--tracers", type=int, default=1)
    ap.add_argument("--parity-levels", action="store_true", help="variable depth (bench.py's flag); default full depth")
    ap.add_argument("--mesh", default="structured", choices=["structured", "delaunay", "delaunay-hilbert"],
                    help="as bench.py: Delaunay triangulation of as many random points as the config has nodes")
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--burst", type=int, default=20)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    variants = [parse_variant(v) for v in a.variants]
    keys = sorted({k for _, env in variants for k in env})
    abi.set_mpi_rank(0, 1)
    abi.set_resident(True)
    if a.mesh == "structured":
        m = synth.config_mesh(a.config, full_depth=not a.parity_levels)  # as bench.py builds it
    else:
        nx, ny, nl = synth.CONFIGS[a.config]
        m = synth.delaunay_mesh(nx * ny, nl, full_depth=not a.parity_levels,
                                numbering="hilbert" if a.mesh == "delaunay-hilbert" else "scipy")
    tracers = synth.make_tracer_fields(m, a.tracers)
    # ONE set of field buffers for every variant (separate allocations differ by up to 6 % in what
    # they stream -- measured with duplicate variants): each variant has its own mesh handles, hence
    # its own plans (cached by handle identity), and the engine is pointed at them in turn
    runs, e = [], None
    for name, env in variants:
        with Knobs(env, keys):
            dm = engine.DeviceMesh(m)
            dm.prepare()
            if e is None:
                e = engine.FctAleBatch(dm, tracers) if a.tracers > 1 else engine.FctAle(dm, tracers[0])
                e.drop_host()  # resident: the library never reads them again (large meshes: host memory)
            e.dm = dm
            for _ in range(3):  # warmup (and the plan, should prepare have missed it)
                assert e.split_pass() == 9, abi.last_error()
            e.sync()
        runs.append((name, env, dm, e))
    del tracers
    times = {name: [] for name, *_ in runs}
    for r in range(a.rounds):
        order = runs if r % 2 == 0 else runs[::-1]
        for name, env, dm, e in order:
            e.dm = dm
            with Knobs(env, keys):
                abi.device_sync()
                t0 = time.perf_counter()
                for _ in range(a.burst):
                    e.split_pass()
                abi.device_sync()
                times[name].append(1e3 * (time.perf_counter() - t0) / a.burst)
    kernels = {}
    for name, env, dm, e in runs:
        e.dm = dm
        with Knobs(env, keys):
            abi.kernel_timing(True)
            abi.kernel_timing_reset()
            for _ in range(a.burst):
                e.split_pass()
            abi.device_sync()
            abi.kernel_timing(False)
            kernels[name] = {k: round(v[1] / max(v[0], 1), 4) for k, v in abi.kernel_stats().items()}
    base = statistics.median(times[runs[0][0]])
    out = {"config": a.config, "tracers": a.tracers, "rounds": a.rounds, "burst": a.burst, "variants": {}}
    for name, env, *_ in runs:
        med = statistics.median(times[name])
        out["variants"][name] = {"env": env, "ms_median": round(med, 4), "ms_min": round(min(times[name]), 4),
                                 "vs_first": round(med / base - 1, 4), "kernels_ms": kernels[name]}
        print(f"{name:28s} {med:8.4f} ms  ({100 * (med / base - 1):+.1f} %)  {kernels[name]}", flush=True)
    print(json.dumps(out))
    e.free()
    for name, env, dm, _ in runs:
        dm.free()


if __name__ == "__main__":
    main()
