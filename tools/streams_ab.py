#!/usr/bin/env python3
"""Tracers on streams against the batch: one mesh, ``--tracers`` single-tracer engines (each with its
own field buffers) whose direction-split passes are spread over 1..N streams, beside the batched
engine (fct_ale_*_batched entries) of the same tracers.  The single engines keep their buffers across
the stream variants (only the stream each engine is driven on changes), so those variants compare
clean; the batch has buffers of its own, and a second batch engine (``batch_b``) shows how far two
allocations of identical work differ.  Every variant's passes alternate in short bursts inside one
process; per variant the median burst over R rounds, in ms per pass of all tracers.

usage: python tools/streams_ab.py [--config '127k x 47'] [--tracers 6] [--streams 1,2,3,6]
           [--rounds 15] [--burst 20]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="127k x 47")
    ap.add_argument("--tracers", type=int, default=6)
    ap.add_argument("--streams", default="1,2,3,6")
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--burst", type=int, default=20)
    a = ap.parse_args()
    abi.set_mpi_rank(0, 1)
    abi.set_resident(True)
    m = synth.config_mesh(a.config, full_depth=True)
    tracers = synth.make_tracer_fields(m, a.tracers)
    dm = engine.DeviceMesh(m)
    dm.prepare()
    batches = [engine.FctAleBatch(dm, tracers) for _ in range(2)]
    singles = [engine.FctAle(dm, f) for f in tracers]
    counts = [int(s) for s in a.streams.split(",")]
    streams = [abi.Stream() for _ in range(max(counts))]
    for e in batches + singles:
        e.drop_host()
    del tracers

    def batch_pass(e):
        def run():
            assert e.split_pass() == 9, abi.last_error()
        return run

    def stream_pass(n):
        def run():
            for k, e in enumerate(singles):
                e.stream = streams[k % n]
                assert e.pre_comm_v() == 7, abi.last_error()
                assert e.post_comm_h() == 9, abi.last_error()
        return run

    variants = [("batch", batch_pass(batches[0]))] + [(f"streams{n}", stream_pass(n)) for n in counts] + \
               [("batch_b", batch_pass(batches[1]))]
    for _, run in variants:  # warmup (plans built on the first pass)
        for _ in range(3):
            run()
    abi.device_sync()
    times = {name: [] for name, _ in variants}
    for r in range(a.rounds):
        for name, run in (variants if r % 2 == 0 else variants[::-1]):
            abi.device_sync()
            t0 = time.perf_counter()
            for _ in range(a.burst):
                run()
            abi.device_sync()
            times[name].append(1e3 * (time.perf_counter() - t0) / a.burst)
    base = statistics.median(times["batch"])
    out = {"config": a.config, "tracers": a.tracers, "rounds": a.rounds, "burst": a.burst, "variants": {}}
    for name, _ in variants:
        med = statistics.median(times[name])
        out["variants"][name] = {"ms_median": round(med, 4), "ms_min": round(min(times[name]), 4),
                                 "vs_batch": round(med / base - 1, 4)}
        print(f"{name:12s} {med:8.4f} ms  ({100 * (med / base - 1):+.1f} %)", flush=True)
    print(json.dumps(out))
    for e in batches + singles:
        e.free()
    dm.free()


if __name__ == "__main__":
    main()
