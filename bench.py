#!/usr/bin/env python3
"""FCT-ALE benchmark: full fct_ale pass (a1..c) through the C-ABI, cell-updates/s and HBM roofline.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 launched by
``torch.distributed.run`` with one rank per GPU.  Rank 0 prints ONE JSON line.

* step      one full pass of the hot path over one batch (one tracer) of synthetic input, split by
            direction (default --path split): fct_ale_pre_comm_v_acc_ (a1..b2 + b3v + cv: the
            vertical half of phase 2 needs only the node's own column) -> fct_ale_post_comm_h_acc_
            (b3h + ch; N > 1: the RCCL halo of fct_plus/fct_minus on a second stream, overlapped
            with the interior edges/nodes).  --path fused: fct_ale_pre_comm_acc_ ->
            fct_ale_post_comm_c_acc_ (or its exchange-overlapped form); --path stepwise: one kernel
            per reference step.
            Device resident: inputs are in HBM before the timed region, no host copies inside it.
* workload  BASELINE.json configs[2]: 1.2M-node x 80-level synthetic mesh (1600 x 750 periodic
            structured triangulation, full depth), 1 tracer, fp64 -- per GPU.  N > 1 is weak scaling:
            the global mesh is 1600 x (750 N) split into N y-strips, each rank owning 1.2M nodes
            (N = 8 is BASELINE configs[4]'s 9.6M-node mesh).
* value     cell-updates/s = (sum over ranks of owned wet cells N_owned x L) / (max-over-ranks time per step).
* roofline  the dominant kernel's algorithmic bytes per launch / its average launch time (HIP events
            on its stream, recorded inside the library around each of its launches in the timed region;
            the other kernels are timed on up to 10 extra steps after it), against 8.0 TB/s.
* check     one more pass on pristine inputs, compared cell for cell with the oracle (per rank on its
            local mesh at N > 1); a mismatch exits with status 1.
* cpu_baseline  the oracle's single-threaded full pass (bit-identical to reference.cpp for a1..b2)
            on the same mesh, rank 0 at N = 1 only; plus "all_cores": P single-threaded oracle
            processes on a P-way strip partition of the same mesh (MPI-style replicas, SURVEY.md
            8(d)), run before this process touches the GPU.

Loads the engine library before torch so the process runs on one HIP runtime; torch is used only
for the multi-rank control plane (gloo: barrier, max-reduce, RCCL unique-id broadcast).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fesom2-accelerate_amd"))

import numpy as np  # noqa: E402

from fesom2_amd import abi, engine, partition, synth  # noqa: E402

HBM_PEAK = 8.0e12  # B/s, MI355X spec (MI355X_MICROARCH.md "Chip-level parameters")
METRIC = "FCT-ALE cell-updates/sec (nodes×levels) at 1/2/4/8 GPUs; % HBM roofline"


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


# ----------------------------------------------------------------------------- algorithmic bytes

def mesh_stats(m):
    """Per-pass unit counts of one local mesh (owned nodes N, L = nl-1)."""
    ln = m.nlev_nod.astype(np.int64) - 1
    cn = int(ln[: m.N].sum())                      # owned wet cells
    cn_halo = int(ln[m.N:].sum())                  # halo wet cells (read by the cluster gathers)
    ce = m.edge_cells                              # sum over edges of max(nl1, nl2)
    # cluster sizes (unique nodes of the elements around each owned node)
    en = m.elem2D_nodes.reshape(-1, 3) - 1
    nie = m.nie.reshape(-1, m.dim)[: m.N] - 1
    # unique cluster nodes per owned node (up to dim*3 candidates, -1 = padding)
    cand = np.where(nie[:, :, None] >= 0, en[np.maximum(nie, 0)], -1).reshape(m.N, -1)
    cand.sort(axis=1)
    prev = np.concatenate([np.full((m.N, 1), -2), cand[:, :-1]], axis=1)
    ring = int(((cand >= 0) & (cand != prev)).sum())
    return dict(N=m.N, E=m.E, T=m.T, cn=cn, cn_halo=cn_halo, ce=ce, ring=ring)


def kernel_bytes(s, ntr=1, split=False):
    """Algorithmic HBM bytes per launch of each kernel of the fused pass (each array element read
    or written once; DESIGN.md §4 derives these).  ntr batched tracers: per-tracer arrays ntr
    times, mesh fields (area_inv; area, hnode, hnode_new) and index arrays once.  split: the
    direction-split pass, where p1v limits the block-internal edges (s["ice"] edge cells, s["nie"]
    edges: their limited fct_adf_h is written by p1v, their raw flux re-read from L2) and b3h runs
    on the other edges."""
    N, E, T, cn, ch, ce, ring = s["N"], s["E"], s["T"], s["cn"], s["cn_halo"], s["ce"], s["ring"]
    ice, nie = (s.get("ice", 0), s.get("nie", 0)) if split else (0, 0)
    cn1 = cn + N  # fct_adf_v columns carry the bottom interface too
    ints_edges = 4 * (N + 1) + 16 * 2 * E      # node->edge CSR (EdgeRef = 16 B, two per edge)
    # p1: ttf, LO (owned + halo, cluster gathers), adf_v, adf_h, plus/minus written; area_inv shared
    p1 = ntr * 8 * (2 * (cn + ch) + cn1 + ce + 2 * cn) + 8 * cn + \
        4 * N + ints_edges + 4 * (N + 1) + 8 * ring + 4 * N
    # b3h: adf_h read + written, plus/minus of both endpoints
    b3h = ntr * 8 * (2 * (ce - ice) + 2 * (cn + ch)) + 16 * (E - nie) + 4 * T
    # p2: plus, minus, adf_v (r + w), del_v (r + w), del_h (r + w), ttf, LO, adf_h; area, hnode,
    # hnode_new shared
    p2 = ntr * 8 * (9 * cn + cn1 + ce) + 8 * 3 * cn + 4 * N + ints_edges
    # p2 with b3h folded in: p2 + the limited adf_h written once (the other endpoint's plus/minus
    # columns are re-reads of arrays p2 already reads)
    p2f = p2 + ntr * 8 * ce
    # split by direction: phase 1 + b3v/cv (adds the limited adf_v write, del_v rw; hnode, hnode_new,
    # area shared), then c-horizontal alone (del_h rw, adf_h; area shared)
    p1v = p1 + ntr * 8 * (cn + 2 * cn + ice) + 8 * 3 * cn + 16 * nie
    p2h = ntr * 8 * (2 * cn + ce) + 8 * cn + 4 * N + ints_edges
    # c-horizontal with b3h folded in: raw adf_h read, limited adf_h written once, plus/minus of both
    # endpoints (owned + halo columns), del_h rw; area shared
    p2hf = ntr * 8 * (2 * cn + 2 * ce + 2 * (cn + ch)) + 8 * cn + 4 * N + ints_edges + 4 * E
    # reference entry sequence in the fast mode: phase 1 + b3v (+ the internal edges) in one kernel
    p1b3v = p1 + ntr * 8 * (cn + ice) + 16 * nie
    # reference entry sequence on the fused kernels: b3v alone (plus/minus, adf_v rw) and the c-step
    # node kernel (cv + ch: del_v, del_h rw; ttf, LO, adf_v, adf_h; area, hnode, hnode_new shared)
    b3v = ntr * 8 * (2 * cn + 2 * cn1) + 4 * N
    c_step = ntr * 8 * (4 * cn + 2 * cn + cn1 + ce) + 8 * 3 * cn + 4 * N + ints_edges
    survey = 32 * cn + ntr * (120 * cn + 24 * ce)  # SURVEY.md §8(d), ints not counted (= 152 Cn + 24 Ce at 1)
    return {"fct_ale_p1": p1, "fct_ale_b3_horizontal": b3h, "fct_ale_p2": p2, "fct_ale_p2_b3h": p2f,
            "fct_ale_p1v": p1v, "fct_ale_p2h": p2h, "fct_ale_p2h_b3h": p2hf,
            "fct_ale_b3_vertical": b3v, "fct_ale_c": c_step, "fct_ale_p1_b3v": p1b3v,
            "pass": p1 + b3h + p2, "pass_fused": p1 + p2f, "pass_split": p1v + b3h + p2h, "survey_pass": survey}


# ----------------------------------------------------------------------------- CPU baselines

def _cpu_replica(job):
    """One MPI-style replica: the oracle's full pass on strip p of P (spawned worker, no GPU)."""
    config, full_depth, P, p, budget = job
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    nx, ny, nl = synth.CONFIGS[config]
    g = synth.make_mesh(nx, ny, nl, full_depth=full_depth)
    m, _ = partition.local_mesh(g, partition.strip_parts(nx, ny, P), p)
    del g
    best, reps = O.time_full_pass(m, synth.make_fields(m), budget_s=budget)
    return int((m.nlev_nod[: m.N].astype(np.int64) - 1).sum()), best, reps


def cpu_all_cores(args, budget=4.0):
    """P concurrent single-threaded oracle processes on a P-way partition of the workload mesh;
    value = all owned cells / the slowest replica's best pass.  P = the cores this process may use,
    at most 16 (the GPU box's CPU share per GPU)."""
    import multiprocessing
    P = max(1, min(16, len(os.sched_getaffinity(0))))
    jobs = [(args.config, not args.parity_levels, P, p, budget) for p in range(P)]
    with multiprocessing.get_context("spawn").Pool(P) as pool:
        res = pool.map(_cpu_replica, jobs)
    cells = sum(r[0] for r in res)
    slowest = max(r[1] for r in res)
    return {"value": round(cells / slowest, 1), "unit": "cell-updates/s", "cores": P,
            "sample": f"{P} concurrent single-threaded oracle processes, y-strip partition of the same "
                      f"{args.config} mesh (one-ring halo each), slowest replica's best of >= "
                      f"{min(r[2] for r in res)} passes ({slowest:.3f} s/pass)"}


def stream_ceiling(args):
    """The chip's streaming rates measured on this GPU right now (tools/stream_probe.hip, a child
    process): a flat 16-B copy, and p1v's own 11-read/4-write stream pattern in its block shape
    without gathers or arithmetic.  None when the probe is not built or fails."""
    import subprocess
    exe = os.path.join(ROOT, "tools", "stream_probe")
    if not os.path.exists(exe):
        return None
    nx, ny, nl = synth.CONFIGS[args.config]
    try:
        out = subprocess.run([exe, str(nx * ny), str(nl - 1), "--json"], capture_output=True, text=True,
                             timeout=120, check=True).stdout
        return json.loads(out.strip().splitlines()[-1])
    except (subprocess.SubprocessError, OSError, ValueError, IndexError):
        return None


def host_info():
    model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), "")
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "usable_cores": len(os.sched_getaffinity(0)), "cpu_model": model}


# ----------------------------------------------------------------------------- workload

def global_dims(args, world):
    """Global mesh: weak scaling stacks `world` copies of the config along y (1.2M nodes per GPU:
    1600 x 6000 = 9.6M at 8 GPUs), strong scaling splits the config itself."""
    nx, ny, nl = synth.CONFIGS[args.config]
    return (nx, ny * world, nl) if args.scaling == "weak" else (nx, ny, nl)


def delaunay(args, npts, nl):
    return synth.delaunay_mesh(npts, nl, full_depth=not args.parity_levels,
                               numbering="hilbert" if args.mesh == "delaunay-hilbert" else "scipy")


def build_local(args, rank, world):
    nx, ny, nl = global_dims(args, world)
    if args.mesh != "structured":
        if world > 1:
            raise SystemExit("--mesh delaunay* is a single-GPU variant")
        return delaunay(args, nx * ny, nl), None
    g = synth.make_mesh(nx, ny, nl, full_depth=not args.parity_levels, name=f"{args.config} x {world}")
    if world == 1:
        return (synth.permute_mesh(g) if args.permuted else g), None
    if args.permuted:
        raise SystemExit("--permuted is a single-GPU stress variant")
    part = partition.strip_parts(nx, ny, world)
    return partition.local_mesh(g, part, rank)  # (local mesh, halo lists)


def host_halo_exchange(dist, lists, cols):
    """FESOM's exchange_nod over gloo for (NT, L) host arrays ``cols`` (owned columns to each
    neighbour, its columns into our halo), in place.  Used by bench's --exchange host step and by the
    per-rank oracle of the parity check (the same exchange test_partition.py checks against the
    single-domain pass)."""
    import torch
    ops, bufs = [], {}
    for q in lists.neighbors:
        out = np.ascontiguousarray(np.stack([a[lists.send[q] - 1] for a in cols]))
        bufs[q] = np.empty((len(cols), lists.recv[q].size) + cols[0].shape[1:])
        ops.append(dist.P2POp(dist.isend, torch.from_numpy(out), q))
        ops.append(dist.P2POp(dist.irecv, torch.from_numpy(bufs[q]), q))
    for w in dist.batch_isend_irecv(ops) if ops else []:
        w.wait()
    for q in lists.neighbors:
        for i, a in enumerate(cols):
            a[lists.recv[q] - 1] = bufs[q][i]


def oracle_local(m, fields, args, dist=None, lists=None):
    """The oracle's pass for every tracer on this rank's local mesh (owned + one-ring halo), with the
    plus/minus halo exchanged over gloo between phase 1 and phase 2 when N > 1 -- FESOM's own
    sequence (docs/refactoring.md:199-200).  Local edges keep the global order, so this equals the
    single-domain pass on every owned cell (tests/test_partition.py)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    out = []
    for fk in fields:
        if args.fct_iter > 1:  # 1 GPU (main() refuses it otherwise)
            out.append(O.iterated_pass(m, fk, args.fct_iter))
            continue
        st, p1 = O.pre_comm(m, fk, vlimit=args.vlimit)
        if st != 5:
            raise RuntimeError(f"oracle pre_comm stopped at alg_state {st}")
        if dist is not None and lists is not None:
            host_halo_exchange(dist, lists, [p1["plus"].reshape(-1, m.L), p1["minus"].reshape(-1, m.L)])
        r = O.post_comm(m, fk, p1["plus"], p1["minus"])
        r.update(plus=p1["plus"], minus=p1["minus"])
        out.append(r)
    return out


def compare_local(m, got, want):
    """Cell-for-cell comparison of one rank's results with its oracle: plus/minus on the owned wet
    cells, del_v/del_h/fct_adf_v on every owned cell, fct_adf_h on every local edge.  Returns
    (mismatch counts per field, max |got - want|, cells compared)."""
    L, nl = m.L, m.nl
    wet = np.arange(L)[None, :] < (m.nlev_nod[: m.N, None].astype(np.int64) - 1)
    bad, max_abs, cells = {}, 0.0, 0
    for k, w in enumerate(want):
        for name, width, rows, mask in (("plus", L, m.N, wet), ("minus", L, m.N, wet), ("del_v", L, m.N, None),
                                        ("del_h", L, m.N, None), ("adf_v", nl, m.N, None),
                                        ("adf_h", L, m.E, None)):
            a = got[name][k][: rows * width].reshape(rows, width)
            b = w[name][: rows * width].reshape(rows, width)
            if mask is not None:
                a, b = a[mask], b[mask]
            diff = a != b
            n = int(np.count_nonzero(diff))
            cells += a.size
            if n:
                bad[name] = bad.get(name, 0) + n
                with np.errstate(invalid="ignore"):
                    d = np.abs(a[diff] - b[diff])
                max_abs = max(max_abs, float(np.nanmax(d)) if np.isfinite(d).any() else float("inf"))
    return bad, max_abs, cells


def verify(args, e, step, m, fields, world, dist, lists, want=None):
    """The reference harness's verify-before-report (kernels/fct_ale_b2.py:97-100, ``answer=``):
    one pass on the pristine inputs, then every rank compares its owned cells (and local edges) with
    the oracle run on its own local mesh -- in parallel on all ranks, the plus/minus halo exchanged
    over gloo for the oracle -- and the counts are summed over ranks.  ``want``: the oracle's outputs
    already computed for cpu_baseline (1 tracer, N = 1)."""
    for name in ("ttf", "LO", "adf_v", "adf_h", "del_v", "del_h", "adf_v2", "adf_h2"):
        if name in e.host:
            e.upload(name)  # the host arrays were never touched in resident mode (adf_*2: zeros)
    step()
    abi.device_sync()
    ntr = len(fields)
    got = {}
    for name, width in (("plus", m.L), ("minus", m.L), ("del_v", m.L), ("del_h", m.L), ("adf_v", m.nl),
                        ("adf_h", m.L)):
        got[name] = e.download(name).reshape(ntr, -1)
    t0 = time.perf_counter()
    if want is None:
        want = oracle_local(m, fields, args, dist if world > 1 else None, lists)
    bad, max_abs, cells = compare_local(m, got, want)
    t_oracle = time.perf_counter() - t0
    if dist is not None:
        import torch
        names = ("plus", "minus", "del_v", "del_h", "adf_v", "adf_h")
        v = torch.tensor([bad.get(k, 0) for k in names] + [cells], dtype=torch.float64)
        dist.all_reduce(v, op=dist.ReduceOp.SUM)
        mx = torch.tensor([max_abs], dtype=torch.float64)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        bad = {k: int(n) for k, n in zip(names, v.tolist()[:-1]) if n}
        cells, max_abs = int(v[-1].item()), float(mx.item())
    return {"exact": not bad, "max_abs": max_abs, "mismatched_cells": bad, "cells_compared": cells,
            "tracers": ntr, "ranks": world, "oracle_s": round(t_oracle, 1),
            "against": ("oracle/fct_ale_oracle.c pass on each rank's local mesh, plus/minus halo exchanged "
                        "over gloo (per tracer)" if world > 1 else
                        "oracle/fct_ale_oracle.c full pass on the same mesh (per tracer)")}


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default=None, choices=list(synth.CONFIGS),
                    help="default: 1.2M x 80 per GPU (weak), 9.6M x 80 in total (strong)")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: the config per GPU; strong: the config split over the GPUs (SURVEY.md 8(e))")
    ap.add_argument("--parity-levels", action="store_true", help="random element levels instead of full depth")
    ap.add_argument("--mesh", default="structured", choices=["structured", "delaunay", "delaunay-hilbert"],
                    help="delaunay: Delaunay triangulation of as many random points as the config has nodes "
                         "(degrees 3..13, scattered numbering; 1 GPU); delaunay-hilbert: the same points "
                         "numbered along a Hilbert curve (the locality of a renumbered FESOM2 mesh)")
    ap.add_argument("--permuted", action="store_true",
                    help="shuffle node/element/edge numbering (unstructured stress variant, 1 GPU)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of oracle passes for cpu_baseline")
    ap.add_argument("--path", default="split", choices=["fused", "split", "stepwise", "reference", "reference-plain"],
                    help="fused: pre_comm + post_comm_c; split: pre_comm_v (+ b3v, cv) + post_comm_h (b3h, ch); "
                         "stepwise: one kernel per reference step; reference: the reference's entry sequence "
                         "pre_comm -> inter_comm -> post_comm -> c in its fast mode (fesom2_set_path_(2): b3v "
                         "and the block-internal edges inside pre_comm); reference-plain: the same sequence without "
                         "the fast mode (what a host that never calls fesom2_set_path_ gets)")
    ap.add_argument("--tracers", type=int, default=1,
                    help="tracers per pass; > 1 uses the batched entry points (BASELINE config 3: 6)")
    ap.add_argument("--graph", action="store_true",
                    help="capture one step into a hipGraph after the warmup and time K replays (no host-side "
                         "work per step; per-kernel timing and roofline are then not available)")
    ap.add_argument("--transfers", action="store_true",
                    help="reference transfer semantics (fesom2_set_resident_(0)): pinned host arrays, the producer's "
                         "H2D of ttf/adf_v/adf_h and every phase's own H2D/D2H inside the timed step, reference entry "
                         "sequence; a PCIe-inclusive rate for DESIGN.md, not the benchmark value (1 GPU, 1 tracer)")
    ap.add_argument("--vlimit", type=int, default=1, choices=[1, 2, 3],
                    help="vertical limiter of a3 (docs/refactoring.md:113-148; reference.cpp has 1 only)")
    ap.add_argument("--fct-iter", type=int, default=1,
                    help="FESOM2's iterative FCT (iter_yn, SURVEY.md 8(f) 1): a step is K-1 rounds of "
                         "pre_comm -> post_comm_iter (LO update, remainder fluxes) then the final pass (--path "
                         "split: the direction-split entries, fused: pre_comm -> post_comm_c); 1 GPU")
    ap.add_argument("--check", action="store_true", default=True,
                    help="(default) after timing, rerun one pass on pristine inputs and compare every owned cell and "
                         "local edge with the oracle on each rank's local mesh; the line carries \"check\" and the "
                         "exit status is 1 on any mismatch")
    ap.add_argument("--kernel-timing", default="dominant", choices=["all", "dominant", "none"],
                    help="HIP events in the timed region around the dominant kernel only (default: the split "
                         "pass's p1v; every other path times every launch), around every launch (all), or none "
                         "(no roofline).  Each timed launch adds two events to the stream: at 127k x 47 timing "
                         "every launch costs 5 %% of the pass.  With 'dominant' the other kernels are timed on "
                         "a few extra steps after the timed region")
    ap.add_argument("--no-check", dest="check", action="store_false", help="skip the parity check")
    ap.add_argument("--exchange", default="rccl", choices=["rccl", "host"],
                    help="N > 1 halo of fct_plus/fct_minus: in-library RCCL (the benchmark), or host copies "
                         "over gloo (validation only: lets N ranks share one GPU, which RCCL refuses)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="measured HBM bytes per launch (rocprofv3 PMC, see profiles/)")
    args = ap.parse_args()
    if args.config is None:
        args.config = "1.2M x 80" if args.scaling == "weak" else "9.6M x 80"

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")

    # all-cores CPU baseline first: its worker processes are spawned before this process touches
    # the GPU
    cpu_all = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_all = cpu_all_cores(args)
        log(f"cpu all cores: {cpu_all}")

    ceiling = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        ceiling = stream_ceiling(args)  # own process, before this one touches the GPU
        log(f"stream ceiling: {ceiling}")

    abi.dll()  # engine first: one HIP runtime for the process
    abi.set_mpi_rank(local_rank, world)  # reference set_mpi_rank_: device = rank % ndev
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        # gloo reports its connections on stdout; the driver reads rank 0's one JSON line there, so
        # fd 1 goes to stderr while the group connects (for good on ranks other than 0)
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        dist.init_process_group("gloo")
        dist.barrier()
        sys.stdout.flush()
        if rank == 0:
            os.dup2(saved, 1)
        os.close(saved)

    t_setup = time.perf_counter()
    m, lists = build_local(args, rank, world)
    if args.tracers > 1 and args.path in ("stepwise", "reference", "reference-plain"):
        raise SystemExit("--tracers > 1 runs the batched (fused or split) entry points only")
    fields = synth.make_tracer_fields(m, args.tracers)
    f = fields[0]
    pinned = []
    if args.transfers:
        if world > 1 or args.tracers > 1 or args.check:
            raise SystemExit("--transfers: 1 GPU, 1 tracer, no --check (outputs land in the input host arrays)")
        args.path = "reference"
        pf = {}
        zeros = np.zeros((m.N + m.H) * m.L)
        for k, v in list(f.items()) + [("plus", zeros), ("minus", zeros)]:
            # page-locked host arrays, as FESOM2 would use allocate_pinned_doubles_
            hp, st = C.c_void_p(), C.c_int(0)
            abi.dll().allocate_pinned_doubles_(C.byref(hp), C.byref(C.c_int(v.size)), C.byref(st))
            a = np.ctypeslib.as_array((C.c_double * v.size).from_address(hp.value))
            a[:] = v
            pf[k] = a
            pinned.append(hp)
        fields = [pf]
        f = pf
    abi.set_resident(not args.transfers)
    abi.set_path({"stepwise": "stepwise", "reference": "reference"}.get(args.path, "fused"))
    dm = engine.DeviceMesh(m)
    dm.prepare()
    mi = dm.info()
    mesh_info = {"ice": mi["internal_edge_cells"], "nie": mi["internal_edges"]}
    if args.fct_iter > 1 and (world > 1 or args.tracers > 1 or args.transfers):
        raise SystemExit("--fct-iter: 1 GPU, 1 tracer, device resident")
    e = engine.FctAle(dm, f, copy=False, vlimit=args.vlimit) if args.tracers == 1 else \
        engine.FctAleBatch(dm, fields, vlimit=args.vlimit)
    if args.path == "reference" and not args.transfers:
        e.bind_c_vertical()  # the fast mode's c-vertical inside pre_comm (fesom2_bind_c_vertical_)
    stream = e.stream

    halo = None
    if world > 1 and args.exchange == "rccl":
        uid = engine.Halo.unique_id() if rank == 0 else (C.c_char * 128)()
        t = torch.frombuffer(bytearray(uid.raw), dtype=torch.uint8).clone()
        dist.broadcast(t, src=0)
        C.memmove(uid, bytes(t.numpy().tobytes()), 128)
        halo = engine.Halo(uid, rank, world, lists, m.nl)
        ci = halo.info()
        log(f"rank {rank}: owned {m.N} halo {m.H} neighbours {lists.neighbors} "
            f"send {[lists.send[q].size for q in lists.neighbors]} recv {[lists.recv[q].size for q in lists.neighbors]} "
            f"rccl {ci}")
        if ci["nranks"] != world or ci["rank"] != rank:
            raise SystemExit(f"RCCL communicator reports rank {ci['rank']} of {ci['nranks']}, expected {rank} of {world}")

    def host_exchange():
        """fct_plus/fct_minus halo through host memory and gloo (--exchange host)."""
        abi.device_sync()
        pm = [e.download(k).reshape(args.tracers, -1, m.L) for k in ("plus", "minus")]
        host_halo_exchange(dist, lists, [a[k] for a in pm for k in range(args.tracers)])
        e.upload("plus", pm[0].reshape(-1))
        e.upload("minus", pm[1].reshape(-1))

    def step_transfers():
        """FESOM2 with the reference's transfer semantics: the producer uploads ttf/adf_v/adf_h
        (src/fesom2-accelerate.cu:269-270), each phase moves its own fields, the host waits after
        phase 1 (where exchange_nod would run) and at the end."""
        import ctypes as C
        for k in ("ttf", "adf_v", "adf_h"):
            abi.dll().transfer_var_async_(e.h[k].ref, abi.arr(e.host[k]), e.stream.ref, C.byref(C.c_bool(True)))
        if e.pre_comm() != 6:
            raise RuntimeError(f"pre_comm: {abi.last_error()}")
        e.sync()
        if (e.inter_comm(), e.post_comm(), e.c_step())[-1] != 9:
            raise RuntimeError(f"phase 2: {abi.last_error()}")
        e.sync()

    def step():
        if args.transfers:
            return step_transfers()
        if args.fct_iter > 1:  # iter_yn: K-1 rounds of phase 1 + iterative phase 2, then the final pass
            s_it = e.iterated_pass(args.fct_iter, final="split" if args.path == "split" else "fused")
            if s_it != 9:
                raise RuntimeError(f"iterated pass alg_state {s_it}: {abi.last_error()}")
            return
        if args.path == "split":
            s1 = e.pre_comm_v()
            if s1 != 7:
                raise RuntimeError(f"pre_comm_v alg_state {s1}: {abi.last_error()}")
            if world > 1 and args.exchange == "host":
                host_exchange()
                s2 = e.post_comm_h()
            else:
                s2 = e.post_comm_h(halo.comm, halo.plan) if halo is not None else e.post_comm_h()
            if s2 != 9:
                raise RuntimeError(f"post_comm_h alg_state {s2}: {abi.last_error()}")
            return
        s1 = e.pre_comm()
        if s1 != 6:
            raise RuntimeError(f"pre_comm alg_state {s1}: {abi.last_error()}")
        if world > 1 and args.exchange == "host":
            host_exchange()
            s2 = e.post_comm_c() if args.path == "fused" else (e.inter_comm(), e.post_comm(), e.c_step())[-1]
        elif args.path in ("stepwise", "reference", "reference-plain"):
            if halo is not None:
                e.exchange(halo.comm, halo.plan)
            s2 = (e.inter_comm(), e.post_comm(), e.c_step())[-1]
        elif halo is not None:
            s2 = e.exchange_post_comm_c(halo.comm, halo.plan)  # exchange overlapped with interior phase 2
        else:
            s2 = e.post_comm_c()
        if s2 != 9:
            raise RuntimeError(f"phase 2 alg_state {s2}: {abi.last_error()}")

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    abi.device_sync()
    setup_s = time.perf_counter() - t_setup

    graph = None
    if args.graph:
        if args.transfers or (world > 1 and args.exchange == "host"):
            raise SystemExit("--graph needs device-resident steps without host exchange")
        abi.device_sync()
        with abi.Graph.capture(stream) as graph:
            step()

        def step():  # noqa: F811 -- the replay replaces the eager step in the timed region
            graph.launch(stream)
        step()
        abi.device_sync()

    # ---- timed region: exactly K steps, barrier + device sync on both sides
    abi.kernel_timing(not args.graph and args.kernel_timing != "none")
    # the split pass's dominant kernel is p1v (an iterated FCT call is dominated by its iteration kernels)
    timed_only = args.kernel_timing == "dominant" and args.path == "split" and args.fct_iter == 1 and not args.graph
    abi.kernel_timing_only("fct_ale_p1v" if timed_only else None)
    abi.kernel_timing_reset()
    barrier()
    abi.device_sync()
    ev0, ev1 = abi.Event(), abi.Event()
    ev0.record(stream)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    abi.device_sync()
    t1 = time.perf_counter()
    barrier()
    abi.kernel_timing(False)
    wall = t1 - t0
    gpu_ms = ev0.elapsed_ms(ev1)
    stats = abi.kernel_stats()
    breakdown = {}
    if timed_only:
        # the per-kernel breakdown, outside the timed region: a few more steps with every launch timed
        # (every rank runs them: the N > 1 step contains the exchange)
        abi.kernel_timing_only(None)
        abi.kernel_timing(True)
        abi.kernel_timing_reset()
        for _ in range(min(args.steps, 10)):
            step()
        abi.device_sync()
        abi.kernel_timing(False)
        breakdown = abi.kernel_stats()

    if dist is not None:
        import torch
        tt = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        wall = float(tt.item())
        cells = torch.tensor([mesh_stats(m)["cn"]], dtype=torch.float64)
        dist.all_reduce(cells, op=dist.ReduceOp.SUM)
        total_cells = float(cells.item())
    else:
        total_cells = float(mesh_stats(m)["cn"])

    ms_step = 1e3 * wall / args.steps
    value = args.tracers * total_cells / (wall / args.steps)  # tracer cell-updates

    # ---- roofline of the dominant kernel (rank-local, all ranks do the same work)
    s = mesh_stats(m)
    s.update(mesh_info)
    kb = kernel_bytes(s, args.tracers, split=args.path in ("split", "reference"))
    per_kernel = {}
    for name, (cnt, tot) in list(stats.items()) + [kv for kv in breakdown.items() if kv[0] not in stats]:
        avg = tot / max(cnt, 1)
        entry = {"launches": cnt, "avg_ms": round(avg, 4),
                 "timed": "timed region" if name in stats else "extra steps after the timed region"}
        if name in kb:
            entry["alg_bytes"] = kb[name]
            entry["GBps"] = round(kb[name] / (avg * 1e-3) / 1e9, 1)
        per_kernel[name] = entry
    dom = max(stats, key=lambda k: stats[k][1]) if stats else None
    traffic = None
    slug = args.config.replace(" ", "").replace(".", "p")  # "127k x 47" -> profiles/traffic_127kx47.json
    for path in (args.traffic, os.path.join(ROOT, "profiles", f"traffic_{slug}.json"),
                 os.path.join(ROOT, "profiles", f"traffic_{slug}_{args.tracers}tr.json")):
        try:
            with open(path) as fh:
                tr = json.load(fh)
        except (OSError, ValueError):
            continue
        if tr.get("workload") == args.config and tr.get("tracers", 1) == args.tracers and \
                args.mesh == "structured" and not args.parity_levels and args.vlimit == 1 and \
                args.fct_iter == 1 and dom in tr.get("bytes_per_launch", {}):
            traffic = tr["bytes_per_launch"][dom]
            break
    roof = None
    if dom in kb:
        avg_s = stats[dom][1] / stats[dom][0] * 1e-3
        achieved = kb[dom] / avg_s / 1e9
        roof = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK / 1e9,
                "unit": "GB/s", "frac": round(achieved / (HBM_PEAK / 1e9), 4), "traffic": traffic,
                "alg_bytes_per_launch": kb[dom], "avg_launch_ms": round(avg_s * 1e3, 4)}
        if ceiling:  # context: what this GPU streams (copy) and streams in p1v's pattern, same run
            roof["stream_ceiling"] = dict(ceiling, frac_of_copy=round(achieved / ceiling["copy_GBps"], 4),
                                          tool="tools/stream_probe.hip")
            if dom == "fct_ale_p1v" and args.tracers == 1:
                roof["stream_ceiling"]["frac_of_p1v_pattern"] = round(achieved / ceiling["p1v_pattern_GBps"], 4)
    pass_gbs = kb["survey_pass"] / (ms_step * 1e-3) / 1e9

    # ---- CPU baseline (rank 0, N = 1 only)
    cpu = None
    oracle_want = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        best, reps, last = O.time_full_pass(m, f, budget_s=args.cpu_budget, keep=True)
        if args.tracers == 1 and args.vlimit == 1 and args.fct_iter == 1 and not args.transfers:
            oracle_want = [last]  # the parity check compares the GPU pass with this very pass
        cpu = {"value": round(s["cn"] / best, 1), "unit": "cell-updates/s", "cores": 1, "kind": "port",
               "sample": f"oracle/fct_ale_oracle.c full pass a1..c (a1..b2 bit-identical to reference.cpp), "
                         f"single thread, same {args.config} mesh, best of {reps} passes ({best:.2f} s/pass)",
               "all_cores": cpu_all, "host": host_info()}
        t_ref = O.time_ref_pre_comm(m, f)
        if t_ref is not None:
            cpu["reference_phase1"] = {
                "value": round(s["cn"] / t_ref, 1), "unit": "cell-updates/s", "cores": 1, "kind": "reference",
                "sample": f"src/reference.cpp fct_ale_a1..a4_reference_ (a1..b2, all the reference runs on the CPU; "
                          f"built from /root/reference by oracle/Makefile), same {args.config} mesh, single thread, "
                          f"best of 2 ({t_ref:.2f} s per phase 1)"}

    check = None
    if args.check and not args.transfers:  # --transfers: outputs land in the input host arrays
        check = verify(args, e, step, m, fields, world, dist, lists, oracle_want)  # a replay when --graph
        log(f"check: {check}")
    if graph is not None:
        graph.free()

    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "cell-updates/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4),
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (deterministic splitmix64 fields, periodic structured triangulation; no dataset)",
            "config": {"workload": f"{args.config} {'parity levels' if args.parity_levels else 'full-depth'}"
                                   + {"structured": "", "delaunay": " Delaunay mesh",
                                      "delaunay-hilbert": " Delaunay mesh, Hilbert numbering"}[args.mesh]
                                   + (" per GPU" if args.scaling == "weak" else f" split over {world} GPU(s)")
                                   + f", {args.tracers} tracer{'s' if args.tracers > 1 else ''}"
                                   + (" (batched)" if args.tracers > 1 else ""),
                       "tracers": args.tracers, "vlimit": args.vlimit, "fct_iterations": args.fct_iter,
                       "nodes_per_gpu": m.N, "levels": m.L,
                       "global_nodes": global_dims(args, world)[0] * global_dims(args, world)[1],
                       "cells_per_gpu": s["cn"], "edge_cells_per_gpu": s["ce"],
                       "parallelism": (f"node partition y-strips x{world}, "
                                       + ("RCCL halo overlapped with interior phase 2" if args.exchange == "rccl"
                                          else "host/gloo halo (validation, not a benchmark)"))
                       if world > 1 else "1 GPU",
                       "path": args.path},
            "roofline": roof,
            "cpu_baseline": cpu,
            "pass_roofline": {"alg_bytes": kb["survey_pass"], "GBps": round(pass_gbs, 1),
                              "frac": round(pass_gbs / (HBM_PEAK / 1e9), 4),
                              "note": "SURVEY.md 8(d) B_pass = 32 Cn + ntracers (120 Cn + 24 Ce) over the whole pass"},
            "kernels": per_kernel,
            "gpu_event_ms_per_step": round(gpu_ms / args.steps, 4),
            "graph": bool(args.graph),
            "transfers": "reference transfer semantics, PCIe inside the timed step" if args.transfers else
                         "device resident (inputs in HBM before the timed region)",
            "setup_s": round(setup_s, 1),
        }
        if check is not None:
            out["check"] = check
        if halo is not None:
            ci = halo.info()
            out["rccl_nranks"] = ci["nranks"]  # ncclCommCount of the communicator the exchange ran on
            out["rccl"] = ci
        print(json.dumps(out), flush=True)

    e.free()
    dm.free()
    for hp in pinned:
        abi.dll().fesom2_free_pinned_(C.byref(hp))
    if halo is not None:
        halo.free()
    if dist is not None:
        dist.destroy_process_group()
    if check is not None and not check["exact"]:
        sys.exit(1)  # a fast wrong answer is not a result


if __name__ == "__main__":
    main()
