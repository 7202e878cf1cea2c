#!/usr/bin/env python3
"""Do two direction-split passes on two HIP streams overlap usefully?

p1v is latency-bound (its own stream pattern runs faster than p1v does) while b3h and p2h stream at
5.6-5.8 TB/s, so a pipeline that runs one pass's (or mesh chunk's) phase 2 beside another's phase 1
could fill the memory pipe better.  This probe measures the ceiling of that idea without any plan
changes: K passes of two independent tracers issued alternately on two streams, against the same
passes on one stream.  Usage (GPU box): python tools/overlap_probe.py [config] [K]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fesom2-accelerate_amd"))

from fesom2_amd import abi, engine, synth  # noqa: E402


def main():
    config = sys.argv[1] if len(sys.argv) > 1 else "1.2M x 80"
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    abi.set_mpi_rank(0, 1)
    abi.set_resident(True)
    nx, ny, nl = synth.CONFIGS[config]
    m = synth.make_mesh(nx, ny, nl, full_depth=True)
    tr = synth.make_tracer_fields(m, 2)
    dm = engine.DeviceMesh(m)
    dm.prepare()
    sa, sb = abi.Stream(), abi.Stream()
    ea = engine.FctAle(dm, tr[0], stream=sa, copy=False)
    eb = engine.FctAle(dm, tr[1], stream=sb, copy=False)

    def run(engines, reps):
        abi.device_sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            for e in engines:
                assert e.pre_comm_v() == 7, abi.last_error()
                assert e.post_comm_h() == 9, abi.last_error()
        abi.device_sync()
        return (time.perf_counter() - t0) * 1e3

    run([ea, eb], 3)  # warm-up
    for rnd in range(3):
        one = run([ea], 2 * K) / (2 * K)
        same = run([ea, ea], K) / (2 * K)
        two = run([ea, eb], K) / (2 * K)
        print(f"round {rnd}: one stream {one:.4f} ms/pass | two tracers, one stream {same:.4f} | "
              f"two streams {two:.4f} ms/pass ({100 * (two / one - 1):+.1f} %)", flush=True)
    ea.free()
    eb.free()
    # batched tracers (BASELINE config 3): one batch of 2T on one stream vs two batches of T on two
    T = int(os.environ.get("OVERLAP_BATCH", "3"))
    if T > 0:
        trs = synth.make_tracer_fields(m, 2 * T)
        whole = engine.FctAleBatch(dm, trs, stream=sa)
        ha = engine.FctAleBatch(dm, trs[:T], stream=sa)
        hb = engine.FctAleBatch(dm, trs[T:], stream=sb)
        run([whole], 2)
        run([ha, hb], 2)
        for rnd in range(3):
            one = run([whole], K // 2) / (K // 2)
            two = run([ha, hb], K // 2) / (K // 2)
            print(f"round {rnd}: {2 * T} tracers batched, one stream {one:.4f} ms/pass | two batches of {T} on two "
                  f"streams {two:.4f} ms/pass ({100 * (two / one - 1):+.1f} %)", flush=True)
        for e in (whole, ha, hb):
            e.free()
    dm.free()


if __name__ == "__main__":
    main()
