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
            the other kernels are timed on up to 10 extra steps after it), against 8.0 TB/s; both byte
            models: the kernel's own (alg_bytes_per_launch -> frac) and SURVEY.md 8(d)'s strict
            minimum for the same work (alg_bytes_min -> frac_min).
* check     one more pass on pristine inputs, compared cell for cell with the oracle: on structured
            meshes by a pool of worker processes (spawned before the GPU is touched), each running
            the oracle on a row strip of the rank's domain widened by one ring (exact without any
            exchange); a mismatch exits with status 1.
* extra     (default --extras auto) further BASELINE configs in the same run, each with its own
            timing, roofline and check: at N = 1 configs[1] (127k x 47, 1 and 6 tracers), configs[3]
            (1.2M x 80, 6 tracers batched), configs[4]'s strong-scaling base (9.6M x 80 on one GPU)
            and one rank's share of its N = 8 point (an interior strip of the 8-way split, no
            exchange), and SURVEY.md 8(d)'s transfer-inclusive rates at 1.2M x 80 (the reference
            transfer semantics; the producer-upload mode with two tracers on two streams), each
            against a same-run PCIe probe; at N > 1 the strong-scaling leg (9.6M x 80 split over
            the N GPUs).  Every N > 1 record carries the per-rank spread of step times and the halo
            exchange's own time and hidden fraction.
* ceilings  pass_roofline.frac_of_copy: the pass's survey bytes per second against a flat 16-B copy
            on this GPU in this run; roofline.frac_of_copy / frac_of_p1v_pattern: the dominant
            kernel's against the copy and against p1v's own stream pattern (one tracer's, or the
            batch's for a batched leg) -- tools/stream_probe.hip, child processes run first.
* cpu_baseline  the oracle's single-threaded full pass (bit-identical to reference.cpp for a1..b2)
            on the same mesh, rank 0 at N = 1 only; plus "per_gpu_share": P single-threaded oracle
            processes on a P-way strip partition of the same mesh (MPI-style replicas, SURVEY.md
            8(d)), run before this process touches the GPU.
* watchdog  a thread per rank: RCCL communicator setup, the first exchange step and each leg have a
            time bound; past it the rank prints its stage to stderr and exits (os._exit, status 3).

Loads the engine library before torch so the process runs on one HIP runtime; torch is used only
for the multi-rank control plane (gloo: barrier, max-reduce, RCCL unique-id broadcast).
"""
from __future__ import annotations

import argparse
import copy
import ctypes as C
import gc
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fesom2-accelerate_amd"))

import numpy as np  # noqa: E402

from fesom2_amd import abi, engine, partition, synth  # noqa: E402

HBM_PEAK = 8.0e12  # B/s, MI355X spec (MI355X_MICROARCH.md "Chip-level parameters")
METRIC = "FCT-ALE cell-updates/sec (nodes×levels) at 1/2/4/8 GPUs; % HBM roofline"
OUTPUTS = (("plus", "L"), ("minus", "L"), ("del_v", "L"), ("del_h", "L"), ("adf_v", "nl"), ("adf_h", "L"))


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
    # split by direction: phase 1 + b3v/cv (adds the limited adf_v write, del_v rw; hnode, hnode_new,
    # area shared), then c-horizontal alone (del_h rw, adf_h; area shared)
    p1v = p1 + ntr * 8 * (cn + 2 * cn + ice) + 8 * 3 * cn + 16 * nie
    p2h = ntr * 8 * (2 * cn + ce) + 8 * cn + 4 * N + ints_edges
    # reference entry sequence in the fast mode: phase 1 + b3v (+ the internal edges) in one kernel
    p1b3v = p1 + ntr * 8 * (cn + ice) + 16 * nie
    # reference entry sequence on the fused kernels: b3v alone (plus/minus, adf_v rw) and the c-step
    # node kernel (cv + ch: del_v, del_h rw; ttf, LO, adf_v, adf_h; area, hnode, hnode_new shared)
    b3v = ntr * 8 * (2 * cn + 2 * cn1) + 4 * N
    c_step = ntr * 8 * (4 * cn + 2 * cn + cn1 + ce) + 8 * 3 * cn + 4 * N + ints_edges
    survey = 32 * cn + ntr * (120 * cn + 24 * ce)  # SURVEY.md §8(d), ints not counted (= 152 Cn + 24 Ce at 1)
    return {"fct_ale_p1": p1, "fct_ale_b3_horizontal": b3h, "fct_ale_p2": p2,
            "fct_ale_p1v": p1v, "fct_ale_p2h": p2h,
            "fct_ale_b3_vertical": b3v, "fct_ale_c": c_step, "fct_ale_p1_b3v": p1b3v,
            "pass": p1 + b3h + p2, "pass_split": p1v + b3h + p2h, "survey_pass": survey}


def pass_roofline(survey_bytes, ms_step, ceiling=None):
    """The whole pass against the HBM peak on SURVEY.md 8(d)'s bytes, and (frac_of_copy) against what
    a flat 16-B copy moves on this GPU in this run (``ceiling``: stream_ceiling's record) -- the
    figure that compares across rounds and boxes."""
    gbs = survey_bytes / (ms_step * 1e-3) / 1e9
    out = {"alg_bytes": survey_bytes, "GBps": round(gbs, 1), "frac": round(gbs / (HBM_PEAK / 1e9), 4),
           "note": "SURVEY.md 8(d) B_pass = 32 Cn + ntracers (120 Cn + 24 Ce) over the whole pass; frac_of_copy: "
                   "the same against a flat 16-B copy on this GPU in this run (tools/stream_probe.hip)"}
    if ceiling and ceiling.get("copy_GBps"):
        out["copy_GBps"] = ceiling["copy_GBps"]
        out["frac_of_copy"] = round(gbs / ceiling["copy_GBps"], 4)
    return out


def reference_byte_models(m):
    """The reference's own per-kernel byte models -- what its kernel_tuner scripts divide by the
    kernel time to print GB/s -- evaluated on this mesh, for the one-kernel-per-step
    path (--path stepwise): a1 `kernels/fct_ale_a1.py:93`, a2 `fct_ale_a2.py:102-111`, a3
    `fct_ale_a3.py:116-149`, b1v `fct_ale_b1_vertical.py:149`, b1h `fct_ale_b1_horizontal.py:70-88`,
    b2 `fct_ale_b2.py:102`, b3v `fct_ale_b3_vertical.py:219`, b3h `fct_ale_b3_horizontal.py:77-100`,
    cv `fct_ale_c_vertical.py:90`, ch `fct_ale_c_horizontal.py:54-70` (fp64)."""
    N, H, T = m.N, m.H, m.T
    ln = m.nlev_nod.astype(np.int64) - 1
    used_all = int(ln.sum())                 # a1 runs over owned + halo nodes
    used = int(ln[:N].sum())
    le = m.nlev_elem.astype(np.int64)
    wet_e = int(np.maximum(le - 1, 0).sum())
    fill_e = int(np.maximum(m.nl - 1 - le, 0).sum())
    nelem = m.nie_num[:N].astype(np.int64)
    a3 = int((4 + ln[:N] * (20 + 20 * nelem) + 32 * ln[:N]).sum())
    t = m.edge_tri.reshape(-1, 2)
    per_edge = int((12 + np.where(t[:, 1] > 0, 8, 4)).sum())
    ce = m.edge_cells
    return {"fct_ale_a1": 4 * (N + H) + 32 * used_all, "fct_ale_a2": 16 * T + 64 * wet_e + 16 * fill_e,
            "fct_ale_a3": a3, "fct_ale_b1_vertical": 4 * N + 32 * used, "fct_ale_b1_horizontal": per_edge + 40 * ce,
            "fct_ale_b2": 4 * N + 56 * used, "fct_ale_b3_vertical": 4 * N + 24 * N + 48 * used,
            "fct_ale_b3_horizontal": per_edge + 48 * ce, "fct_ale_c_vertical": 4 * N + 72 * used,
            "fct_ale_c_horizontal": per_edge + 56 * ce}


def kernel_bytes_min(s, ntr=1):
    """SURVEY.md 8(d)'s strict minimum bytes for the work of the phase-1 kernels (each array of its
    table read or written once, no index arrays, no halo columns, no internal-edge flux writes):
    phase 1 = ttf, LO, adf_v, area_inv read + plus/minus written = 48 Cn, + adf_h read 8 Ce; p1v
    adds the vertical half of phase 2 (limited adf_v written, del_v read + written, hnode,
    hnode_new, area read) = 48 Cn.  Mesh fields (area_inv; area, hnode, hnode_new) count once per
    batch: p1 = 8 Cn + ntr (40 Cn + 8 Ce), p1v = 32 Cn + ntr (64 Cn + 8 Ce) (96 Cn + 8 Ce at 1)."""
    cn, ce = s["cn"], s["ce"]
    return {"fct_ale_p1": 8 * cn + ntr * (40 * cn + 8 * ce),
            "fct_ale_p1v": 32 * cn + ntr * (64 * cn + 8 * ce)}


_CODE_OBJECT = []


def engine_code_object():
    """Code-object hash of the engine library this process runs (fesom2_amd._paths.code_object_hash)."""
    if not _CODE_OBJECT:
        from fesom2_amd import _paths
        _CODE_OBJECT.append(_paths.code_object_hash())
    return _CODE_OBJECT[0]


def traffic_paths(args):
    """The traffic files that may hold this workload's PMC bytes: --traffic, then
    profiles/traffic_<config>[_<T>tr | _rank<R>of<N>].json ("127k x 47" -> traffic_127kx47.json)."""
    slug = args.config.replace(" ", "").replace(".", "p")
    em = getattr(args, "emulate", None)
    if em:
        return [args.traffic, os.path.join(ROOT, "profiles", f"traffic_{slug}_rank{em[0]}of{em[1]}.json")]
    return [args.traffic, os.path.join(ROOT, "profiles", f"traffic_{slug}.json"),
            os.path.join(ROOT, "profiles", f"traffic_{slug}_{args.tracers}tr.json")]


def find_traffic(args, world, dom, code=None):
    """PMC bytes per launch of kernel `dom` for this workload, and where they came from.  A file
    matches on workload, tracer count and emulated rank; its bytes are reported only when its
    `code_object` stamp equals the loaded library's (the kernels it measured are the ones that ran),
    else traffic is None and the info says `traffic_stale` (a kernel change without a new PMC pass)."""
    em = getattr(args, "emulate", None)
    if args.mesh != "structured" or args.parity_levels or args.vlimit != 1 or args.fct_iter != 1 or \
            args.transfers or not (args.scaling == "weak" or world == 1):
        return None, {}
    for path in traffic_paths(args):
        try:
            with open(path) as fh:
                tr = json.load(fh)
        except (OSError, ValueError):
            continue
        if tr.get("workload") != args.config or tr.get("tracers", 1) != args.tracers or \
                tr.get("emulate") != (f"{em[0]}/{em[1]}" if em else None) or \
                dom not in tr.get("bytes_per_launch", {}):
            continue
        code = code or engine_code_object()
        info = {"traffic_source": os.path.relpath(path, ROOT), "traffic_code_object": tr.get("code_object"),
                "code_object": code}
        if tr.get("code_object") != code:
            info["traffic_stale"] = True
            return None, info
        return tr["bytes_per_launch"][dom], info
    return None, {}


# ----------------------------------------------------------------------------- worker pool

def _worker_init():
    """Pool workers are single-threaded (the OpenMP field generator too): the pool is the parallelism."""
    os.environ["OMP_NUM_THREADS"] = "1"


def make_pool(world):
    """Worker processes for the CPU baselines and the parity check, spawned before this process
    touches the GPU (they never do): 16 per rank (the GPU box's CPU share per GPU), fewer when the
    cores this rank may use, shared by the node's ranks, hold less."""
    import multiprocessing
    n = len(os.sched_getaffinity(0))
    P = max(1, min(16, n // world if n >= 16 * world else n))
    return multiprocessing.get_context("spawn").Pool(P, initializer=_worker_init), P


# ----------------------------------------------------------------------------- CPU baselines

def _cpu_replica(job):
    """One MPI-style replica: the oracle's full pass on strip p of P (spawned worker, no GPU)."""
    config, full_depth, P, p, budget = job
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    nx, ny, nl = synth.CONFIGS[config]
    y0, y1 = partition.strip_rows(ny, P, p)
    m, _ = partition.strip_local_mesh(nx, ny, nl, y0, y1, full_depth=full_depth)
    best, reps = O.time_full_pass(m, synth.make_fields(m), budget_s=budget)
    return int((m.nlev_nod[: m.N].astype(np.int64) - 1).sum()), best, reps


def cpu_per_gpu_share(args, pool, P, budget=4.0):
    """P concurrent single-threaded oracle processes on a P-way partition of the workload mesh --
    P = this GPU's share of the host's cores (16 of a 128-core, 8-GPU node; the worker pool's size,
    make_pool) -- plus the whole host extrapolated linearly from them (the replicas share nothing, so
    the full node would run physical_cores of them at the same per-core rate; not measured here: the
    GPU box's other seven GPUs' jobs own the other cores).  value = all owned cells / the slowest
    replica's best pass."""
    jobs = [(args.config, not args.parity_levels, P, p, budget) for p in range(P)]
    res = pool.map(_cpu_replica, jobs)
    cells = sum(r[0] for r in res)
    slowest = max(r[1] for r in res)
    value = cells / slowest
    phys = host_info()["physical_cores"]
    return {"value": round(value, 1), "unit": "cell-updates/s", "cores": P,
            "represents": f"this GPU's share of the host: {P} of {phys or '?'} physical cores, one MPI-style "
                          f"oracle replica per core",
            "sample": f"{P} concurrent single-threaded oracle processes, y-strip partition of the same "
                      f"{args.config} mesh (one-ring halo each), slowest replica's best of >= "
                      f"{min(r[2] for r in res)} passes ({slowest:.3f} s/pass)",
            "full_host_estimate": {"value": round(value * phys / P, 1) if phys else None, "cores": phys,
                                   "unit": "cell-updates/s",
                                   "method": f"per-core rate of the {P} measured replicas x the host's physical "
                                             f"cores (linear: independent replicas; an estimate, not measured)"}}


def stream_ceiling(config, tracers=0):
    """The chip's streaming rates measured on this GPU right now (tools/stream_probe.hip, a child
    process) at ``config``'s size: a flat 16-B copy, p1v's own 11-read/4-write stream pattern in its
    block shape without gathers or arithmetic (odd L: its slot shape), and with ``tracers`` > 1 (even
    L) the batched pattern of the batched plan's 6-column blocks, tiles tracer-fastest
    (``batch_GBps[str(tracers)]``).  None when the probe is not built or fails."""
    import subprocess
    exe = os.path.join(ROOT, "tools", "stream_probe")
    if not os.path.exists(exe):
        return None
    nx, ny, nl = synth.CONFIGS[config]
    try:
        cmd = [exe, str(nx * ny), str(nl - 1), "--json"] + ([str(tracers)] if tracers > 1 else [])
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=180, check=True).stdout
        lines = [json.loads(ln) for ln in out.strip().splitlines() if ln.startswith("{")]
        res = dict(lines[-1])
        res["batch_GBps"] = {str(d["tracers"]): d["batch_GBps"] for d in lines[:-1]
                             if d.get("G") == 6 and d.get("order") == "tracer-fastest"}
        res["config"] = config
        return res
    except (subprocess.SubprocessError, OSError, ValueError, IndexError, KeyError):
        return None


def host_info():
    model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), "")
    except OSError:
        pass
    phys = set()
    try:
        with open("/proc/cpuinfo") as fh:
            pid = cid = None
            for ln in fh:
                if ln.startswith("physical id"):
                    pid = ln.split(":", 1)[1].strip()
                elif ln.startswith("core id"):
                    cid = ln.split(":", 1)[1].strip()
                elif not ln.strip():
                    if cid is not None:
                        phys.add((pid, cid))
                    pid = cid = None
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "physical_cores": len(phys) or None,
            "usable_cores": len(os.sched_getaffinity(0)), "cpu_model": model}


# ----------------------------------------------------------------------------- watchdog

class Watchdog:
    """Bounds the stages that can stall a multi-rank run without a diagnosis (RCCL communicator
    setup, the first exchange, a whole leg): past the bound the rank prints its stage and exits
    with status 3 (os._exit: no re-exec, no cleanup that could block on the stalled collective).
    ``on_fire`` (rank 0) may print what was measured so far first."""

    def __init__(self, rank):
        self.rank, self.stage, self.deadline, self.bound = rank, None, None, 0.0
        self.on_fire = None
        self.lock = threading.Lock()
        threading.Thread(target=self._loop, daemon=True, name="bench-watchdog").start()

    def arm(self, stage, seconds):
        with self.lock:
            self.stage, self.bound, self.deadline = stage, seconds, time.monotonic() + seconds

    def disarm(self):
        with self.lock:
            self.stage = self.deadline = None

    def _loop(self):
        while True:
            time.sleep(0.5)
            with self.lock:
                late = self.deadline is not None and time.monotonic() > self.deadline
                stage, bound = self.stage, self.bound
            if late:
                log(f"rank {self.rank}: watchdog: stage '{stage}' not done within {bound:.0f} s -- exiting")
                try:
                    if self.on_fire:
                        self.on_fire(stage)
                finally:
                    sys.stderr.flush()
                    sys.stdout.flush()
                    os._exit(3)


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
    """This rank's local mesh (owned y-strip + one-ring halo, built from the strip alone:
    partition.strip_local_mesh) and its exchange lists."""
    em = getattr(args, "emulate", None)
    if em:  # one rank's strip of a world-way strong split, on this single GPU (halo from global ids)
        if world > 1 or args.scaling != "strong" or args.mesh != "structured" or args.permuted:
            # (its check regenerates the strips in natural order: a permuted numbering would mismatch)
            raise SystemExit("--emulate-rank: 1 GPU, --scaling strong, structured mesh, natural numbering")
        rank, world = em
    nx, ny, nl = global_dims(args, world)
    if args.mesh != "structured":
        if world > 1:
            raise SystemExit("--mesh delaunay* is a single-GPU variant")
        return delaunay(args, nx * ny, nl), None
    name = f"{args.config} x {world}" if args.scaling == "weak" else f"{args.config} / {world}"
    if world == 1:
        g = synth.make_mesh(nx, ny, nl, full_depth=not args.parity_levels, name=name)
        return (synth.permute_mesh(g) if args.permuted else g), None
    if args.permuted:
        raise SystemExit("--permuted is a single-GPU stress variant")
    y0, y1 = partition.strip_rows(ny, world, rank)
    row_part = (np.arange(ny) * world) // ny
    return partition.strip_local_mesh(nx, ny, nl, y0, y1, full_depth=not args.parity_levels, row_part=row_part,
                                      rank=rank, name=f"{name}[rank {rank}]")


def host_halo_exchange(dist, lists, cols):
    """FESOM's exchange_nod over gloo for (NT, L) host arrays ``cols`` (owned columns to each
    neighbour, its columns into our halo), in place.  Used by bench's --exchange host step and by the
    per-rank oracle of the serial parity check (the same exchange test_partition.py checks against
    the single-domain pass)."""
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


def _compare(bad, name, a, b, acc):
    """Count differing cells of a vs b into bad[name]; acc = [max_abs, cells]."""
    diff = a != b
    n = int(np.count_nonzero(diff))
    acc[1] += a.size
    if n:
        bad[name] = bad.get(name, 0) + n
        with np.errstate(invalid="ignore"):
            d = np.abs(a[diff] - b[diff])
        acc[0] = max(acc[0], float(np.nanmax(d)) if np.isfinite(d).any() else float("inf"))


def compare_local(m, got, want):
    """Cell-for-cell comparison of one rank's results with its oracle: plus/minus on the owned wet
    cells, del_v/del_h/fct_adf_v on every owned cell, fct_adf_h on every local edge.  Returns
    (mismatch counts per field, max |got - want|, cells compared)."""
    L, nl = m.L, m.nl
    wet = np.arange(L)[None, :] < (m.nlev_nod[: m.N, None].astype(np.int64) - 1)
    bad, acc = {}, [0.0, 0]
    for k, w in enumerate(want):
        for name, width, rows, mask in (("plus", L, m.N, wet), ("minus", L, m.N, wet), ("del_v", L, m.N, None),
                                        ("del_h", L, m.N, None), ("adf_v", nl, m.N, None),
                                        ("adf_h", L, m.E, None)):
            a = got[name][k][: rows * width].reshape(rows, width)
            b = w[name][: rows * width].reshape(rows, width)
            if mask is not None:
                a, b = a[mask], b[mask]
            _compare(bad, name, a, b, acc)
    return bad, acc[0], acc[1]


def _check_strip(job):
    """Parallel parity check, one worker job: the oracle on rows [a, b) of rank rows [R0, R1) of the
    structured nx x ny mesh, compared with the rank's GPU outputs (memory-mapped files).

    The oracle runs on the strip widened by one row on each side as owned nodes (plus their
    one-ring halo): every node of rows [a-1, b] then has its whole cluster and all of its edges, so
    its plus/minus are final without an exchange, and so are the b3-limited fluxes and the c-step of
    rows [a, b).  Node sums keep the global edge order, hence the comparison is cell-for-cell exact.
    Edges are compared by the strip of their smallest rank-owned endpoint (each local edge once)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    nx, ny, nl, full, vlimit, (R0, R1), (a, b), ntr, (mode, src) = job
    L = nl - 1
    e0, e1 = strip_edge_range(nx, ny, R0, R1, a, b)
    y0, y1 = max(0, a - 1), min(ny, b + 1)
    m, _ = partition.strip_local_mesh(nx, ny, nl, y0, y1, full_depth=full)
    n0, n1 = (a - y0) * nx, (b - y0) * nx        # rows [a, b) in the widened strip
    g0 = (a - R0) * nx                           # ... and in the rank's owned numbering
    ends = m.node_gid[m.edges.reshape(-1, 2) - 1]
    owned = (ends >= R0 * nx) & (ends < R1 * nx)
    key = np.where(owned, ends, np.iinfo(np.int64).max).min(axis=1)
    tgt = (key >= a * nx) & (key < b * nx)
    gpu_e = partition.strip_edge_index(nx, ny, R0, R1, m.edge_gid[tgt])
    if not np.array_equal(gpu_e, np.arange(e0, e1)):
        raise RuntimeError(f"strip rows {a}:{b}: its edges are not the rank's edges {e0}:{e1}")
    wet = np.arange(L)[None, :] < (m.nlev_nod[n0:n1, None].astype(np.int64) - 1)
    if mode == "files":  # the rank's whole arrays, memory-mapped: this strip's rows / edges of them
        mm = {k: np.memmap(path, dtype=np.float64, mode="r", shape=shape) for k, (path, shape) in src.items()}
        rows = lambda name, k, wd: mm[name][k][g0 * wd:(g0 + n1 - n0) * wd]
        edges = lambda k: mm["adf_h"][k].reshape(-1, L)[e0:e1]
    else:  # "data": the strip's rows / edges, sent with the job
        rows = lambda name, k, wd: src[name][k]
        edges = lambda k: src["adf_h"][k].reshape(-1, L)
    bad, acc = {}, [0.0, 0]
    for k in range(ntr):
        f = synth.make_fields(m, seed=43 + k)
        if k:  # one ocean state: the mesh fields of every tracer are the first one's (make_tracer_fields)
            f0 = synth.make_fields(m, seed=43)
            for name in ("area", "area_inv", "hnode", "hnode_new"):
                f[name] = f0[name]
        st, p1 = O.pre_comm(m, f, vlimit=vlimit)
        if st != 5:
            raise RuntimeError(f"oracle pre_comm stopped at alg_state {st}")
        w = O.post_comm(m, f, p1["plus"], p1["minus"])
        w.update(plus=p1["plus"], minus=p1["minus"])
        for name, width in OUTPUTS:
            wd = L if width == "L" else nl
            if name == "adf_h":
                _compare(bad, name, edges(k), w[name].reshape(-1, wd)[tgt], acc)
                continue
            ga = rows(name, k, wd).reshape(-1, wd)
            wa = w[name][n0 * wd:n1 * wd].reshape(-1, wd)
            if name in ("plus", "minus"):
                ga, wa = ga[wet], wa[wet]
            _compare(bad, name, ga, wa, acc)
    return bad, acc[0], acc[1]


def strip_edge_range(nx, ny, R0, R1, a, b):
    """[e0, e1): the rank's local edges (owned rows [R0, R1)) that _check_strip compares for rows
    [a, b) -- contiguous, since an edge's smallest rank-owned endpoint lies in the row it starts in
    (or in row R0 for the vertical/diagonal edges coming up from row R0 - 1, which lead the list)."""
    first_of = lambda j: int(partition.strip_edge_index(nx, ny, R0, R1, [3 * nx * j])[0])
    total = first_of(R1 - 1) + (nx if R1 - 1 == ny - 1 else 3 * nx)
    return (0 if a == R0 else first_of(a)), (total if b == R1 else first_of(b))


def pristine(m, name, ntr):
    """The pristine input `name` of all ntr tracers (tracer-slowest, as the batched handles hold
    them), regenerated from the synthetic generator."""
    if ntr == 1:
        return synth.make_field(m, name, seed=43)
    return np.concatenate([synth.make_field(m, name, seed=43 + k) for k in range(ntr)])


def run_check_pass(args, e, step, m, ntr):
    """One pass on pristine inputs (the outputs the timed steps overwrote are uploaded again)."""
    for name in ("adf_v", "adf_h", "del_v", "del_h"):
        e.upload(name, pristine(m, name, ntr))
    step()
    abi.device_sync()


def verify_parallel(args, ctx, e, step, m, world, rank, check_pass=None, fetch=None):
    """The reference harness's verify-before-report (kernels/fct_ale_b2.py:97-100, ``answer=``) for the
    structured meshes: one pass on pristine inputs, the outputs downloaded into memory-mapped files,
    then ctx.pool's workers check row strips of this rank's domain (_check_strip); counts are summed
    over the strips and over the ranks.  ``check_pass()`` replaces the default pristine pass and
    ``fetch(name, out)`` the download of all tracers' output ``name`` (the transfer legs: outputs in
    the host arrays); an emulated rank (args.emulate = (rank, world), one GPU) checks its strip."""
    ntr = args.tracers
    em = getattr(args, "emulate", None)
    if em:
        rank, world = em
    nx, ny, nl = global_dims(args, world)
    R0, R1 = partition.strip_rows(ny, world, rank) if world > 1 else (0, ny)
    if check_pass is not None:
        check_pass()
    else:
        run_check_pass(args, e, step, m, ntr)
    if fetch is None:
        fetch = lambda name, out: e.download(name, out=out)
    # strips of about 80k nodes (a few seconds of oracle work each), at least one per worker
    rows = R1 - R0
    nstrip = max(min(rows, ctx.nworkers), min(rows, -(-(rows * nx) // 80000)))
    cuts = [R0 + (rows * s_) // nstrip for s_ in range(nstrip + 1)]
    strips = [(cuts[s_], cuts[s_ + 1]) for s_ in range(nstrip) if cuts[s_ + 1] > cuts[s_]]
    # the outputs reach the workers as memory-mapped files in /dev/shm when it has room for every
    # rank's (no copy), else as the strips' slices sent with the jobs
    sizes = {name: ntr * e.size(name) // e.ntr for name, _ in OUTPUTS}
    need = sum(8 * max(sizes[name], 1) for name, _ in OUTPUTS)
    shm = "/dev/shm"
    try:
        st_ = os.statvfs(shm)
        use_files = st_.f_bavail * st_.f_frsize >= 1.5 * need * world
    except OSError:
        use_files = False
    files, paths = {}, []
    t0 = time.perf_counter()
    try:
        if use_files:
            import tempfile
            for name, _ in OUTPUTS:
                n = sizes[name]
                fd, path = tempfile.mkstemp(prefix=f"f2a_check_{os.getpid()}_{name}_", dir=shm)
                os.close(fd)
                paths.append(path)
                buf = np.memmap(path, dtype=np.float64, mode="w+", shape=(max(n, 1),))
                fetch(name, buf)
                buf.flush()
                del buf
                files[name] = (path, (ntr, n // ntr))
            srcs = [("files", files)] * len(strips)
        else:
            host = {}
            for name, _ in OUTPUTS:
                host[name] = np.empty(max(sizes[name], 1))
                fetch(name, host[name])
                host[name] = host[name][: sizes[name]].reshape(ntr, -1)
            srcs = []
            for a, b in strips:
                e0, e1 = strip_edge_range(nx, ny, R0, R1, a, b)
                d = {}
                for name, width in OUTPUTS:
                    wd = m.L if width == "L" else m.nl
                    d[name] = host[name][:, e0 * wd:e1 * wd] if name == "adf_h" else \
                        host[name][:, (a - R0) * nx * wd:(b - R0) * nx * wd]
                srcs.append(("data", d))
        jobs = [(nx, ny, nl, not args.parity_levels, args.vlimit, (R0, R1), st, ntr, src)
                for st, src in zip(strips, srcs)]
        res = ctx.pool.map(_check_strip, jobs, chunksize=1)
    finally:
        for p in paths:
            try:
                os.unlink(p)
            except OSError:
                pass
    t_oracle = time.perf_counter() - t0
    bad, max_abs, cells = {}, 0.0, 0
    for b_, mx, c in res:
        for k, v in b_.items():
            bad[k] = bad.get(k, 0) + v
        max_abs, cells = max(max_abs, mx), cells + c
    bad, max_abs, cells = reduce_check(ctx, bad, max_abs, cells)
    return {"exact": not bad, "max_abs": max_abs, "mismatched_cells": bad, "cells_compared": cells,
            "tracers": ntr, "ranks": world, "oracle_s": round(t_oracle, 1),
            "against": f"oracle/fct_ale_oracle.c on {len(jobs)} row strips per rank, each widened by one ring "
                       f"(exact without an exchange), {ctx.nworkers} worker processes per rank (per tracer); "
                       f"outputs {'memory-mapped from /dev/shm' if use_files else 'sent with the jobs'}"}


def reduce_check(ctx, bad, max_abs, cells):
    if ctx.dist is None:
        return bad, max_abs, cells
    import torch
    dist = ctx.dist
    names = [k for k, _ in OUTPUTS]
    v = torch.tensor([bad.get(k, 0) for k in names] + [cells], dtype=torch.float64)
    dist.all_reduce(v, op=dist.ReduceOp.SUM)
    mx = torch.tensor([max_abs], dtype=torch.float64)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    return {k: int(n) for k, n in zip(names, v.tolist()[:-1]) if n}, float(mx.item()), int(v[-1].item())


def verify(args, ctx, e, step, m, fields, world, lists, want=None):
    """The serial verify-before-report (unstructured / permuted meshes, iter_yn, or the headline at
    N = 1 where cpu_baseline's oracle pass is reused): one pass on the pristine inputs, then every
    rank compares its owned cells (and local edges) with the oracle run on its own local mesh -- in
    parallel on all ranks, the plus/minus halo exchanged over gloo for the oracle.  ``want``: the
    oracle's outputs already computed for cpu_baseline (1 tracer, N = 1)."""
    for name in ("ttf", "LO", "adf_v", "adf_h", "del_v", "del_h", "adf_v2", "adf_h2"):
        if name in e.host:
            e.upload(name)  # the host arrays were never touched in resident mode (adf_*2: zeros)
    step()
    abi.device_sync()
    ntr = len(fields)
    got = {name: e.download(name).reshape(ntr, -1) for name, _ in OUTPUTS}
    t0 = time.perf_counter()
    if want is None:
        want = oracle_local(m, fields, args, ctx.dist if world > 1 else None, lists)
    bad, max_abs, cells = compare_local(m, got, want)
    t_oracle = time.perf_counter() - t0
    bad, max_abs, cells = reduce_check(ctx, bad, max_abs, cells)
    return {"exact": not bad, "max_abs": max_abs, "mismatched_cells": bad, "cells_compared": cells,
            "tracers": ntr, "ranks": world, "oracle_s": round(t_oracle, 1),
            "against": ("oracle/fct_ale_oracle.c pass on each rank's local mesh, plus/minus halo exchanged "
                        "over gloo (per tracer)" if world > 1 else
                        "oracle/fct_ale_oracle.c full pass on the same mesh (per tracer)")}


# ----------------------------------------------------------------------------- PCIe / halo helpers

def pcie_probe(nbytes=1 << 30, reps=5):
    """What this box's PCIe link moves between page-locked host memory and HBM, through the
    library's own transfer entries: H2D (transfer_var_, synchronous), D2H (fesom2_download_ into a
    pinned array) and both directions at once (transfer_var_async_ and fesom2_transfer_back_async_
    on two streams), 1 GiB each, best of ``reps``."""
    n = nbytes // 8
    bufs, hps, hs, ss = [], [], [], []
    try:
        for _ in range(2):
            a, hp = abi.pinned(n)
            hps.append(hp)
            a[:] = 1.0
            h = abi.Handle("pcie")
            abi.check(abi.alloc_var(h, a), "alloc_var_(pcie)")
            bufs.append(a)
            hs.append(h)
        ss += [abi.Stream(), abi.Stream()]
        s1, s2 = ss

        def best(fn):
            t = []
            for _ in range(reps):
                abi.device_sync()
                t0 = time.perf_counter()
                fn()
                abi.device_sync()
                t.append(time.perf_counter() - t0)
            return min(t)

        st = C.c_int(0)
        h2d = best(lambda: abi.dll().transfer_var_(hs[0].ref, abi.arr(bufs[0])))
        d2h = best(lambda: abi.dll().fesom2_download_(hs[0].ref, abi.arr(bufs[0]), C.byref(st)))

        def duplex():
            abi.transfer_var_async(hs[0], bufs[0], s1)
            abi.transfer_back_async(hs[1], bufs[1], s2)
        dup = best(duplex)
        return {"h2d_GBps": round(nbytes / h2d / 1e9, 2), "d2h_GBps": round(nbytes / d2h / 1e9, 2),
                "duplex_GBps_each_way": round(nbytes / dup / 1e9, 2), "bytes": nbytes,
                "method": "1 GiB page-locked (allocate_pinned_doubles_) <-> one handle: transfer_var_ (H2D), "
                          "fesom2_download_ (D2H), transfer_var_async_ + fesom2_transfer_back_async_ on two "
                          f"streams at once (duplex); best of {reps}"}
    finally:
        # on every path: the transfers done, then the handles and streams, then the pinned arrays
        # the handles point at (an error half-way must not leak 2 GiB of HBM into the later legs)
        abi.device_sync()
        for h in hs:
            abi.dll().fesom2_free_(h.ref)
        for s_ in ss:
            abi.dll().fesom2_free_stream_(s_.ref)
        for hp in hps:
            abi.free_pinned(hp)


def oracle_halo_plus_minus(nx, ny, nl, full_depth, vlimit, world, rank):
    """plus/minus of the halo rows of rank's strip of the world-way y-strip split of the nx x ny
    structured mesh (rows y0 - 1 and y1) from the oracle on those rows alone (each a one-row strip
    with its own one-ring halo: exact), (H, L) in the local halo order -- what the exchange would
    deliver; the emulated-rank leg's check uses it (tests/test_bench.py checks it against the
    single-domain pass)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    y0, y1 = partition.strip_rows(ny, world, rank)
    rows = ([y0 - 1] if y0 > 0 else []) + ([y1] if y1 < ny else [])
    L = nl - 1
    plus, minus = np.zeros((len(rows) * nx, L)), np.zeros((len(rows) * nx, L))
    for k, j in enumerate(rows):
        mh, _ = partition.strip_local_mesh(nx, ny, nl, j, j + 1, full_depth=full_depth)
        st, p1 = O.pre_comm(mh, synth.make_fields(mh), vlimit=vlimit)
        if st != 5:
            raise RuntimeError(f"oracle pre_comm (halo row {j}) stopped at alg_state {st}")
        plus[k * nx:(k + 1) * nx] = p1["plus"][: nx * L].reshape(nx, L)
        minus[k * nx:(k + 1) * nx] = p1["minus"][: nx * L].reshape(nx, L)
    return plus, minus


def single_pass_baseline(args, m, dm, batch_ms):
    """A batched leg's tracers the way the reference takes them: one tracer per call
    (`src/fesom2-accelerate.cu:258-379`), each its own buffers, their direction-split passes in
    sequence on one stream -- warmup, then ``args.steps`` sequences, wall time between device syncs.
    Distinct tracers: six repeats of ONE tracer would find the previous pass's tail in the Infinity
    Cache, which a sequence of different tracers does not (profiles/r06/s23)."""
    stream = abi.Stream()
    engines, shared = [], None
    try:
        for k in range(args.tracers):
            fk = synth.make_fields(m, seed=43 + k)  # the fields make_tracer_fields gives tracer k
            if shared is None:
                shared = {n: fk[n] for n in ("area", "area_inv", "hnode", "hnode_new")}
            fk.update(shared)
            e = engine.FctAle(dm, fk, stream=stream, vlimit=args.vlimit, copy=False)
            e.drop_host()
            engines.append(e)
            del fk

        def sequence():
            for e in engines:
                s1 = e.pre_comm_v()
                s2 = e.post_comm_h() if s1 == 7 else s1
                if s2 != 9:
                    raise RuntimeError(f"single-tracer pass alg_state {s2}: {abi.last_error()}")

        for _ in range(max(1, args.warmup)):
            sequence()
        abi.device_sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            sequence()
        abi.device_sync()
        ms = 1e3 * (time.perf_counter() - t0) / args.steps
    finally:
        for e in engines:
            e.free()
        stream.free()
    return {"ms_per_step": round(ms, 4), "batch_gain": round(batch_ms / ms - 1, 4),
            "note": f"the same {args.tracers} tracers as single-tracer split passes (pre_comm_v -> post_comm_h) in "
                    f"sequence, each tracer its own buffers, one stream, {args.steps} sequences after "
                    f"{max(1, args.warmup)} of warmup; batch_gain = batch ms / this - 1"}


# ----------------------------------------------------------------------------- one leg

class Ctx:
    """Per-process run state: rank, world, gloo group, worker pool, watchdog."""
    rank = 0
    world = 1
    dist = None
    pool = None
    nworkers = 0
    watchdog = None
    pcie = None  # pcie_probe(), once per run (the transfer legs)

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def allgather(self, values):
        """[per rank: list of floats] over the gloo group."""
        if self.dist is None:
            return [list(values)]
        import torch
        t = torch.tensor(values, dtype=torch.float64)
        out = [torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [o.tolist() for o in out]


def run_leg(args, ctx, headline=False, cpu_all=None, ceiling=None):
    """Build, warm up, time K steps, break the kernels down, check.  Returns the leg's record."""
    rank, world, dist = ctx.rank, ctx.world, ctx.dist
    if args.transfers and ctx.pcie is None:
        ctx.pcie = pcie_probe()
        log(f"pcie probe: {ctx.pcie}")
    t_setup = time.perf_counter()
    m, lists = build_local(args, rank, world)
    if args.tracers > 1 and args.path in ("stepwise", "reference", "reference-plain"):
        raise SystemExit("--tracers > 1 runs the batched (fused or split) entry points only")
    fields = synth.make_tracer_fields(m, args.tracers)
    f = fields[0]
    pinned = []
    mode = args.transfers  # None (device resident), "reference" or "producer" (host transfers in the step)
    # the fields a transfer step moves per tracer: the producer's (fct_ale_muscl_LH's) ttf, LO,
    # fct_adf_v, fct_adf_h and the host-accumulated del_ttf_advvert / del_ttf_advhoriz; with the
    # reference semantics also fct_plus/fct_minus (the host's exchange_nod round trip)
    streamed = ("ttf", "LO", "adf_v", "adf_h", "del_v", "del_h")
    if mode:
        if world > 1 or getattr(args, "emulate", None) or args.mesh != "structured" or args.fct_iter > 1 or \
                args.permuted:  # (its check regenerates the strips in natural order)
            raise SystemExit("--transfers: 1 GPU, structured mesh in natural numbering, one FCT iteration")
        if mode == "reference" and args.tracers != 1:
            raise SystemExit("--transfers reference: 1 tracer (the reference's entries take one)")
        if mode == "producer" and args.tracers != 2:
            raise SystemExit("--transfers producer: 2 tracers, one stream each")
        args.path = "reference" if mode == "reference" else "split"
        if mode == "reference":
            streamed += ("plus", "minus")
        pfs = []
        for fk in fields:
            pf = dict(fk)
            for k in streamed:
                v = fk[k] if k in fk else np.zeros((m.N + m.H) * m.L)
                a, hp = abi.pinned(v.size)  # page-locked, as FESOM2 would use allocate_pinned_doubles_
                a[:] = v
                pf[k] = a
                pinned.append(hp)
            pfs.append(pf)
        fields = pfs
        f = fields[0]
    abi.set_resident(mode != "reference")
    abi.set_path({"stepwise": "stepwise", "reference": "reference"}.get(args.path, "fused"))
    dm = engine.DeviceMesh(m)
    dm.prepare()
    mi = dm.info(batched=args.tracers > 1 and mode != "producer")
    mesh_info = {"ice": mi["internal_edge_cells"], "nie": mi["internal_edges"]}
    # the plan the kernels ran on: p1v block columns, block-internal edges, cluster unions
    plan_info = {"p1v_columns": mi["p1v_columns"], "internal_edges": mi["internal_edges"],
                 "union_columns": mi.get("union_columns", 0), "union_max": mi.get("union_max", 0)}
    order = dm.pass_order(args.tracers if mode != "producer" else 1)  # the Infinity-Cache pass order
    if args.fct_iter > 1 and (world > 1 or args.tracers > 1 or mode):
        raise SystemExit("--fct-iter: 1 GPU, 1 tracer, device resident")
    if mode == "producer":  # one single-tracer engine (and stream) per tracer
        engines = [engine.FctAle(dm, fk, copy=False, vlimit=args.vlimit) for fk in fields]
        e = engines[0]
    else:
        e = engine.FctAle(dm, f, copy=False, vlimit=args.vlimit) if args.tracers == 1 else \
            engine.FctAleBatch(dm, fields, vlimit=args.vlimit)
        engines = [e]
    parallel_check = (args.check and ctx.pool is not None and args.mesh == "structured" and not args.permuted
                      and args.fct_iter == 1)
    cpu_leg = headline and rank == 0 and world == 1 and not args.no_cpu_baseline
    if parallel_check and not cpu_leg and not mode:
        # the check regenerates its pristine inputs: no second host copy of the fields (the
        # transfer legs keep theirs: the step uploads from them)
        e.drop_host()
        del fields, f
        fields = f = None
        gc.collect()
    if args.path == "reference" and not args.transfers:
        e.bind_c_vertical()  # the fast mode's c-vertical inside pre_comm (fesom2_bind_c_vertical_)
    stream = e.stream

    halo = None
    if world > 1 and args.exchange == "rccl":
        import torch
        uid = engine.Halo.unique_id() if rank == 0 else (C.c_char * 128)()
        t = torch.frombuffer(bytearray(uid.raw), dtype=torch.uint8).clone()
        dist.broadcast(t, src=0)
        C.memmove(uid, bytes(t.numpy().tobytes()), 128)
        ctx.watchdog.arm(f"{args.leg}: RCCL communicator setup (ncclCommInitRank)", args.comm_timeout)
        halo = engine.Halo(uid, rank, world, lists, m.nl)
        ci = halo.info()
        ctx.watchdog.disarm()
        log(f"rank {rank}: {args.leg}: owned {m.N} halo {m.H} neighbours {lists.neighbors} "
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
        (src/fesom2-accelerate.cu:269-270) and the host's del_ttf_advvert/advhoriz, each phase moves
        its own fields (pre_comm: LO up, plus/minus down, :268, :337-339; inter_comm: adf_v down,
        :354-355; post_comm: plus/minus up, adf_h down, :364-365, :377-378; c-step: del_ttf down),
        the host waits after phase 1 (where exchange_nod would run) and at the end."""
        for k in ("ttf", "adf_v", "adf_h", "del_v", "del_h"):
            abi.transfer_var_async(e.h[k], e.host[k], e.stream, k in ("ttf", "adf_v", "adf_h"))
        if e.pre_comm() != 6:
            raise RuntimeError(f"pre_comm: {abi.last_error()}")
        e.sync()
        if (e.inter_comm(), e.post_comm(), e.c_step())[-1] != 9:
            raise RuntimeError(f"phase 2: {abi.last_error()}")
        e.sync()

    def step_producer():
        """Device-resident split pass of two tracers, each on its own stream, with the host's uploads
        of the producer's fields and the download of del_ttf inside the step: tracer 1's uploads
        overlap tracer 0's pass and tracer 0's downloads; the host waits for both at the end."""
        for ek in engines:
            for k in streamed:
                abi.transfer_var_async(ek.h[k], ek.host[k], ek.stream, k in ("ttf", "adf_v", "adf_h"))
            s1 = ek.pre_comm_v()
            if s1 != 7:
                raise RuntimeError(f"pre_comm_v alg_state {s1}: {abi.last_error()}")
            s2 = ek.post_comm_h()
            if s2 != 9:
                raise RuntimeError(f"post_comm_h alg_state {s2}: {abi.last_error()}")
            for k in ("del_v", "del_h"):
                abi.transfer_back_async(ek.h[k], ek.host[k], ek.stream)
        for ek in engines:
            ek.sync()

    def step():
        if mode == "reference":
            return step_transfers()
        if mode == "producer":
            return step_producer()
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

    # the first step carries the first exchange: bounded on every rank (a stalled RCCL send/recv)
    if world > 1:
        ctx.watchdog.arm(f"{args.leg}: first step (first halo exchange)", args.comm_timeout)
        step()
        abi.device_sync()
        ctx.barrier()
        ctx.watchdog.disarm()
    for _ in range(args.warmup):
        step()
    abi.device_sync()
    setup_s = time.perf_counter() - t_setup

    graph = None
    if args.graph:
        if mode or (world > 1 and args.exchange == "host"):
            raise SystemExit("--graph needs device-resident steps without host exchange")
        abi.device_sync()
        with abi.Graph.capture(stream) as graph:
            step()

        def step():  # noqa: F811 -- the replay replaces the eager step in the timed region
            graph.launch(stream)
        step()
        abi.device_sync()

    # ---- timed region: exactly K steps, barrier + device sync on both sides
    timing = not args.graph and args.kernel_timing != "none" and not mode  # transfer legs: wall time only
    # the split pass's dominant kernel is p1v (an iterated FCT call is dominated by its iteration kernels)
    timed_only = args.kernel_timing == "dominant" and args.path == "split" and args.fct_iter == 1 and not args.graph
    abi.kernel_timing_only("fct_ale_p1v" if timed_only else None)
    abi.kernel_timing_reset()
    # the dominant kernel's events on every --timing-every'th step of the timed region (a sample:
    # each event pair costs a small partition's pass ~2 %; switching does not synchronise)
    every = max(1, args.timing_every) if timed_only else 1
    ctx.barrier()
    abi.device_sync()
    ev0, ev1 = abi.Event(), abi.Event()
    ev0.record(stream)
    t0 = time.perf_counter()
    for i in range(args.steps):
        abi.kernel_timing(timing and i % every == 0)
        step()
    ev1.record(stream)
    abi.device_sync()
    t1 = time.perf_counter()
    ctx.barrier()
    abi.kernel_timing(False)
    wall_rank = t1 - t0
    gpu_ms = ev0.elapsed_ms(ev1)
    ev0.free()
    ev1.free()
    stats = abi.kernel_stats()
    breakdown = {}
    if timed_only or world > 1:
        # the per-kernel breakdown (and at N > 1 the halo exchange's own time and its exposed wait),
        # outside the timed region: a few more steps with every launch timed (every rank runs them:
        # the N > 1 step contains the exchange)
        abi.kernel_timing_only(None)
        abi.kernel_timing(True)
        abi.kernel_timing_reset()
        for _ in range(min(args.steps, 10)):
            step()
        abi.device_sync()
        abi.kernel_timing(False)
        breakdown = abi.kernel_stats()
        ctx.barrier()

    s = mesh_stats(m)
    s.update(mesh_info)
    # per-rank spread (max over ranks is the step time) and the exchange's own timing
    avg = lambda st, k: st[k][1] / st[k][0] if k in st and st[k][0] else 0.0
    per_rank = ctx.allgather([1e3 * wall_rank / args.steps, avg(stats, "fct_ale_p1v"),
                              avg(breakdown, "halo_exchange"), avg(breakdown, "halo_wait"), float(s["cn"])])
    wall = max(r[0] for r in per_rank) * args.steps / 1e3
    total_cells = sum(r[4] for r in per_rank)
    ms_step = 1e3 * wall / args.steps
    value = args.tracers * total_cells / (wall / args.steps)  # tracer cell-updates

    # ---- roofline of the dominant kernel (rank-local, all ranks do the same work)
    kb = kernel_bytes(s, args.tracers, split=args.path in ("split", "reference"))
    kbm = kernel_bytes_min(s, args.tracers)
    per_kernel = {}
    refm = reference_byte_models(m) if args.path == "stepwise" and args.tracers == 1 else None
    for name, (cnt, tot) in list(stats.items()) + [kv for kv in breakdown.items() if kv[0] not in stats]:
        a_ms = tot / max(cnt, 1)
        entry = {"launches": cnt, "avg_ms": round(a_ms, 4),
                 "timed": "timed region" if name in stats else "extra steps after the timed region"}
        if name in kb:
            entry["alg_bytes"] = kb[name]
            entry["GBps"] = round(kb[name] / (a_ms * 1e-3) / 1e9, 1)
        if refm and name in refm:  # the reference harness's own bandwidth figure for this kernel
            entry["ref_model_bytes"] = refm[name]
            entry["ref_model_GBps"] = round(refm[name] / (a_ms * 1e-3) / 1e9, 1)
        per_kernel[name] = entry
    dom = max(stats, key=lambda k: stats[k][1]) if stats else None
    traffic, traffic_info = find_traffic(args, world, dom)
    roof = None
    if dom in kb:
        avg_s = stats[dom][1] / stats[dom][0] * 1e-3
        achieved = kb[dom] / avg_s / 1e9
        roof = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK / 1e9,
                "unit": "GB/s", "frac": round(achieved / (HBM_PEAK / 1e9), 4), "traffic": traffic,
                "alg_bytes_per_launch": kb[dom], "avg_launch_ms": round(avg_s * 1e3, 4),
                "byte_model": "alg_bytes_per_launch: the kernel's own arrays, halo columns, internal-edge "
                              "flux writes and index arrays once each (DESIGN.md 3)"}
        if dom in kbm:
            roof["alg_bytes_min"] = kbm[dom]
            roof["frac_min"] = round(kbm[dom] / avg_s / HBM_PEAK, 4)
            roof["byte_model_min"] = "alg_bytes_min: SURVEY.md 8(d)'s strict minimum for the same work " \
                                     "(p1v: 32 Cn + ntracers (64 Cn + 8 Ce); p1: 8 Cn + ntracers (40 Cn + 8 Ce))"
        roof.update(traffic_info)
        if traffic:
            roof["traffic_over_alg"] = round(traffic / kb[dom], 3)
        if ceiling:  # context: what this GPU streams (copy) and streams in p1v's pattern, same run
            roof["stream_ceiling"] = dict(ceiling, tool="tools/stream_probe.hip")
            roof["frac_of_copy"] = round(achieved / ceiling["copy_GBps"], 4)
            # p1v's own stream pattern (no gathers): one tracer's, or the batch's (tracer-fastest tiles
            # of the plan's block size) for a batched call
            pat = ceiling.get("p1v_pattern_GBps") if args.tracers == 1 else \
                ceiling.get("batch_GBps", {}).get(str(args.tracers))
            if dom == "fct_ale_p1v" and pat:
                roof["frac_of_p1v_pattern"] = round(achieved / pat, 4)
                roof["p1v_pattern_GBps"] = pat

    # ---- CPU baseline (rank 0, N = 1, headline only)
    cpu = None
    oracle_want = None
    if cpu_leg:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        best, reps, last = O.time_full_pass(m, f, budget_s=args.cpu_budget, keep=True)
        if args.tracers == 1 and args.vlimit == 1 and args.fct_iter == 1 and not args.transfers:
            oracle_want = [last]  # the parity check compares the GPU pass with this very pass
        cpu = {"value": round(s["cn"] / best, 1), "unit": "cell-updates/s", "cores": 1, "kind": "port",
               "sample": f"oracle/fct_ale_oracle.c full pass a1..c (a1..b2 bit-identical to reference.cpp), "
                         f"single thread, same {args.config} mesh, best of {reps} passes ({best:.2f} s/pass)",
               "per_gpu_share": cpu_all, "host": host_info()}
        t_ref = O.time_ref_pre_comm(m, f)
        if t_ref is not None:
            cpu["reference_phase1"] = {
                "value": round(s["cn"] / t_ref, 1), "unit": "cell-updates/s", "cores": 1, "kind": "reference",
                "sample": f"src/reference.cpp fct_ale_a1..a4_reference_ (a1..b2, all the reference runs on the CPU; "
                          f"built from /root/reference by oracle/Makefile), same {args.config} mesh, single thread, "
                          f"best of 2 ({t_ref:.2f} s per phase 1)"}

    check = None
    em = getattr(args, "emulate", None)
    if args.check:
        if mode:
            # the transfer legs: pristine inputs into the host arrays the step uploads, one step, then
            # the outputs where the host gets them (the reference semantics: every output comes back
            # to the host arrays; producer mode: del_ttf on the host, the rest on the device)
            host_out = set(streamed) if mode == "reference" else {"del_v", "del_h"}

            def transfer_check_pass():
                for k, ek in enumerate(engines):
                    for name in streamed:
                        if name in ("plus", "minus"):
                            ek.host[name][:] = 0.0
                        else:
                            ek.host[name][:] = synth.make_field(m, name, seed=43 + k)
                step()
                abi.device_sync()

            def transfer_fetch(name, out):
                n = e.size(name)
                for k, ek in enumerate(engines):
                    out[k * n:(k + 1) * n] = ek.host[name][:n] if name in host_out else ek.download(name)

            check = verify_parallel(args, ctx, e, step, m, world, rank, check_pass=transfer_check_pass,
                                    fetch=transfer_fetch)
        elif em:
            # one strip of the strong split without an exchange in its timed steps: the check pass
            # takes the halo plus/minus the exchange would deliver from the oracle (halo rows only)
            hp_, hm_ = oracle_halo_plus_minus(*global_dims(args, em[1]), not args.parity_levels, args.vlimit,
                                              em[1], em[0])

            def emulated_check_pass():
                for name in ("adf_v", "adf_h", "del_v", "del_h"):
                    e.upload(name, pristine(m, name, 1))
                s1 = e.pre_comm_v()
                if s1 != 7:
                    raise RuntimeError(f"pre_comm_v alg_state {s1}: {abi.last_error()}")
                e.sync()
                for name, halo_vals in (("plus", hp_), ("minus", hm_)):
                    a = e.download(name).reshape(-1, m.L)
                    a[m.N:m.N + m.H] = halo_vals
                    e.upload(name, a.reshape(-1))
                s2 = e.post_comm_h()
                if s2 != 9:
                    raise RuntimeError(f"post_comm_h alg_state {s2}: {abi.last_error()}")
                abi.device_sync()

            check = verify_parallel(args, ctx, e, step, m, world, rank, check_pass=emulated_check_pass)
            check["halo"] = "plus/minus of the two halo rows from the oracle (what the exchange delivers)"
        elif parallel_check and oracle_want is None:
            check = verify_parallel(args, ctx, e, step, m, world, rank)  # a replay when --graph
        else:
            check = verify(args, ctx, e, step, m, fields, world, lists, oracle_want)
        log(f"check ({args.leg}): {check}")
    if graph is not None:
        graph.free()
    # the same tracers as the reference calls them, one tracer per call in sequence (batched
    # device-resident legs on one GPU; after the timed region and the check)
    singles = None
    if args.tracers > 1 and not mode and world == 1 and not em and args.fct_iter == 1 and args.path == "split" \
            and not args.graph and not getattr(args, "no_single_baseline", False):
        singles = single_pass_baseline(args, m, dm, ms_step)
        log(f"single-tracer passes ({args.leg}): {singles}")

    # the whole pass's figures also inside `roofline` (the driver's parsed record keeps that object
    # whole; pass_roofline stays beside it): frac of 8 TB/s and of this run's copy rate
    pr = pass_roofline(kb["survey_pass"], ms_step, ceiling)
    if roof is not None:
        roof["pass_frac"] = pr["frac"]
        if "frac_of_copy" in pr:
            roof["pass_frac_of_copy"] = pr["frac_of_copy"]
    rec = {"value": round(value, 1), "ms_per_step": round(ms_step, 4), "roofline": roof,
           "pass_roofline": pr,
           "kernels": per_kernel, "gpu_event_ms_per_step": round(gpu_ms / args.steps, 4),
           "setup_s": round(setup_s, 1), "cpu": cpu, "check": check, "m": m, "s": s,
           "pass_order": order, "plan": plan_info}
    if singles:
        rec["single_passes"] = singles
    if world > 1:
        ms = [r[0] for r in per_rank]
        rec["ranks"] = {
            "ms_per_step": [round(x, 4) for x in ms], "ms_per_step_min": round(min(ms), 4),
            "ms_per_step_max": round(max(ms), 4), "spread": round(max(ms) / min(ms) - 1, 4) if min(ms) else None,
            "p1v_avg_ms": [round(r[1], 4) for r in per_rank],
            "halo_exchange_ms": [round(r[2], 4) for r in per_rank],
            "halo_wait_ms": [round(r[3], 4) for r in per_rank],
            "halo_hidden_frac": [round(max(0.0, min(1.0, 1 - r[3] / r[2])), 4) if r[2] else None for r in per_rank],
            "timing": "ms_per_step: timed region per rank (value uses the max); halo_exchange_ms: pack + grouped "
                      "RCCL send/recv + unpack on the halo stream, halo_wait_ms: the compute stream's wait for it "
                      "after the interior work (the exposed part), both from HIP events on extra steps after the "
                      "timed region"}
    if halo is not None:
        ci = halo.info()
        rec["rccl_nranks"] = ci["nranks"]  # ncclCommCount of the communicator the exchange ran on
        rec["rccl"] = ci
    if mode:
        # PCIe traffic of one step (both tracers in producer mode) and its rate against the same
        # run's probe of the link (ctx.pcie, measured once before the first transfer leg)
        NT, L, nl, E = m.N + m.H, m.L, m.nl, m.E
        per = {"ttf": NT * L, "LO": NT * L, "del_v": NT * L, "del_h": NT * L, "plus": NT * L, "minus": NT * L,
               "adf_v": NT * nl, "adf_h": E * L}
        if mode == "reference":
            up = [*streamed]                                          # producer's + LO + plus/minus (post_comm)
            down = ["plus", "minus", "adf_v", "adf_h", "del_v", "del_h"]
        else:
            up, down = list(streamed), ["del_v", "del_h"]
        h2d = 8 * len(engines) * sum(per[k] for k in up)
        d2h = 8 * len(engines) * sum(per[k] for k in down)
        sec = ms_step * 1e-3
        pc = ctx.pcie or {}
        rec["transfers"] = {
            "mode": {"reference": "reference transfer semantics: pre_comm -> inter_comm -> post_comm -> c_acc_, "
                                  "every phase's own H2D/D2H (src/fesom2-accelerate.cu:268, :337-339, :354-355, "
                                  ":364-365, :377-378), fast mode, the producer's uploads inside the step",
                     "producer": "device-resident split pass, per tracer on its own stream: the producer's "
                                 "uploads (ttf, LO, fct_adf_v, fct_adf_h, del_ttf in) and del_ttf out inside the "
                                 "step, two tracers overlapped"}[mode],
            "h2d_bytes_per_step": h2d, "d2h_bytes_per_step": d2h,
            "h2d_GBps": round(h2d / sec / 1e9, 2), "d2h_GBps": round(d2h / sec / 1e9, 2),
            "h2d_frac_of_probe": round(h2d / sec / 1e9 / pc["h2d_GBps"], 3) if pc.get("h2d_GBps") else None,
            "d2h_frac_of_probe": round(d2h / sec / 1e9 / pc["d2h_GBps"], 3) if pc.get("d2h_GBps") else None,
            # both directions at the probe's duplex rate at once: the step's floor on this link
            "pcie_floor_ms": round(1e3 * max(h2d, d2h) / (pc["duplex_GBps_each_way"] * 1e9), 2)
            if pc.get("duplex_GBps_each_way") else None,
            "probe": pc}
    for ek in engines[1:]:
        ek.free()
    e.free()
    dm.free()
    for hp in pinned:
        abi.dll().fesom2_free_pinned_(C.byref(hp))
    if halo is not None:
        halo.free()
    return rec


def workload_name(args, world, m):
    return (f"{args.config} {'parity levels' if args.parity_levels else 'full-depth'}"
            + {"structured": "", "delaunay": " Delaunay mesh", "delaunay-hilbert": " Delaunay mesh, Hilbert numbering"}[args.mesh]
            + (" per GPU" if args.scaling == "weak" else f" split over {world} GPU(s)")
            + f", {args.tracers} tracer{'s' if args.tracers > 1 else ''}" + (" (batched)" if args.tracers > 1 else ""))


def extra_legs(args, world):
    """The further BASELINE configs measured in the same run (--extras auto)."""
    strong = ("config4_strong_" + args.strong_config.replace(" ", "").replace(".", "p"),
              dict(config=args.strong_config, tracers=1, scaling="strong"))
    if world == 1:
        # the small partition's legs time at least ~0.1 s (a 20-step region of 0.28 ms passes is
        # 6 ms, where the clocks' ramp after setup still shows)
        return [("config1_127kx47", dict(config="127k x 47", tracers=1, scaling="weak",
                                         steps=max(args.steps, 400), warmup=max(args.warmup, 20))),
                ("config1_127kx47_6tracers", dict(config="127k x 47", tracers=6, scaling="weak",
                                                  steps=max(args.steps, 80), warmup=max(args.warmup, 10))),
                ("config3_1p2Mx80_6tracers", dict(config="1.2M x 80", tracers=6, scaling="weak")),
                strong,
                # BASELINE configs[4]'s N = 8 point, one rank's share: an interior strip (two neighbours)
                # of the 8-way strong split, 3200 x 375 rows = 1.2M nodes, on this GPU
                (strong[0].replace("config4_strong_", "config4_strong_rank3of8_"),
                 dict(strong[1], emulate=(3, 8))),
                # SURVEY.md 8(d)'s transfer-inclusive rates at 1.2M x 80 (PCIe inside the step)
                ("config2_transfers_reference", dict(config="1.2M x 80", tracers=1, scaling="weak",
                                                     transfers="reference", steps=min(args.steps, 10),
                                                     warmup=min(args.warmup, 2))),
                ("config2_transfers_producer_2tracers", dict(config="1.2M x 80", tracers=2, scaling="weak",
                                                             transfers="producer", steps=min(args.steps, 10),
                                                             warmup=min(args.warmup, 2)))]
    return [strong]


def select_legs(legs, spec):
    """The extra legs --legs names (comma-separated; None: all of them, in their order)."""
    if not spec:
        return legs
    want = set(spec.split(","))
    unknown = want - {n for n, _ in legs}
    if unknown:
        raise SystemExit(f"--legs: unknown {sorted(unknown)}; known {[n for n, _ in legs]}")
    return [(n, o) for n, o in legs if n in want]


def compact(rec, args, world):
    """An extra leg's sub-record."""
    m, s = rec["m"], rec["s"]
    out = {"workload": workload_name(args, world, m), "scaling": args.scaling, "value": rec["value"],
           "unit": "cell-updates/s" if args.tracers == 1 else "tracer-cell-updates/s",
           "ms_per_step": rec["ms_per_step"], "steps": args.steps, "warmup": args.warmup,
           "nodes_per_gpu": m.N, "levels": m.L, "cells_per_gpu": s["cn"], "tracers": args.tracers,
           "roofline": rec["roofline"], "pass_roofline": rec["pass_roofline"],
           "kernels_ms": {k: v["avg_ms"] for k, v in rec["kernels"].items()}, "check": rec["check"],
           "setup_s": rec["setup_s"], "pass_order": rec["pass_order"], "plan": rec.get("plan")}
    for k in ("ranks", "rccl_nranks", "transfers", "single_passes"):
        if k in rec:
            out[k] = rec[k]
    if getattr(args, "emulate", None):
        out["emulated_rank"] = {"rank": args.emulate[0], "of": args.emulate[1],
                                "note": "one strip of the strong split on this GPU (halo from global ids), no "
                                        "exchange in the timed steps: the per-rank compute of that N-GPU point"}
    return out


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
    ap.add_argument("--no-single-baseline", action="store_true",
                    help="batched legs: skip timing the same tracers as single-tracer passes in sequence")
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
    ap.add_argument("--transfers", nargs="?", const="reference", default=None, choices=["reference", "producer"],
                    help="PCIe inside the timed step, pinned host arrays (1 GPU): 'reference' (the default of the bare "
                         "flag) the reference transfer semantics (fesom2_set_resident_(0), the reference entry sequence, "
                         "every phase's own H2D/D2H, the producer's uploads; 1 tracer); 'producer' the device-resident "
                         "split pass with only the producer's uploads and del_ttf's download in the step, two tracers "
                         "on two streams (--tracers 2).  A PCIe-inclusive rate, not the benchmark value")
    ap.add_argument("--emulate-rank", default=None,
                    help="R/N: time rank R's strip of an N-way --scaling strong split on this one GPU (halo from "
                         "global ids, no exchange in the timed steps; the check takes the halo plus/minus from the "
                         "oracle): the per-rank compute of the N-GPU point")
    ap.add_argument("--vlimit", type=int, default=1, choices=[1, 2, 3],
                    help="vertical limiter of a3 (docs/refactoring.md:113-148; reference.cpp has 1 only)")
    ap.add_argument("--fct-iter", type=int, default=1,
                    help="FESOM2's iterative FCT (iter_yn, SURVEY.md 8(f) 1): a step is K-1 rounds of "
                         "pre_comm -> post_comm_iter (LO update, remainder fluxes) then the final pass (--path "
                         "split: the direction-split entries, fused: pre_comm -> post_comm_c); 1 GPU")
    ap.add_argument("--check", action="store_true", default=True,
                    help="(default) after timing, rerun one pass on pristine inputs and compare every owned cell and "
                         "local edge with the oracle; the line carries \"check\" and the exit status is 1 on any "
                         "mismatch")
    ap.add_argument("--kernel-timing", default="dominant", choices=["all", "dominant", "none"],
                    help="HIP events in the timed region around the dominant kernel only (default: the split "
                         "pass's p1v; every other path times every launch), around every launch (all), or none "
                         "(no roofline).  Each timed launch adds two events to the stream: at 127k x 47 timing "
                         "every launch costs 5 %% of the pass.  With 'dominant' the other kernels are timed on "
                         "a few extra steps after the timed region")
    ap.add_argument("--timing-every", type=int, default=4,
                    help="with --kernel-timing dominant: bracket the dominant kernel of every k-th timed step "
                         "(a sample of K/k launches; 1: every step)")
    ap.add_argument("--no-check", dest="check", action="store_false", help="skip the parity check")
    ap.add_argument("--exchange", default="rccl", choices=["rccl", "host"],
                    help="N > 1 halo of fct_plus/fct_minus: in-library RCCL (the benchmark), or host copies "
                         "over gloo (validation only: lets N ranks share one GPU, which RCCL refuses)")
    ap.add_argument("--extras", default="auto", choices=["auto", "on", "none"],
                    help="auto (default): with the default workload also measure the other BASELINE configs in "
                         "this run (N = 1: 127k x 47 with 1 and 6 tracers, 1.2M x 80 with 6 tracers, 9.6M x 80 on "
                         "one GPU; N > 1: 9.6M x 80 split over the N GPUs) as 'extra' sub-records; on: whatever the "
                         "headline workload (e.g. with --exchange host, to rehearse N > 1 on one GPU)")
    ap.add_argument("--legs", default=None,
                    help="comma-separated names of the extra legs to run (default: all of them)")
    ap.add_argument("--strong-config", default="9.6M x 80", choices=list(synth.CONFIGS),
                    help="the strong-scaling leg's global mesh (BASELINE configs[4]: 9.6M x 80)")
    ap.add_argument("--comm-timeout", type=float, default=180.0,
                    help="watchdog bound (s) of RCCL communicator setup and of the first exchange step")
    ap.add_argument("--leg-timeout", type=float, default=420.0,
                    help="watchdog bound (s) of each extra leg (the 9.6M x 80 leg on one GPU takes about 60 s)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="measured HBM bytes per launch (rocprofv3 PMC, see profiles/)")
    args = ap.parse_args()
    if args.emulate_rank:
        r_, n_ = (int(v) for v in args.emulate_rank.split("/"))
        if not (0 <= r_ < n_ and n_ > 1):
            raise SystemExit("--emulate-rank R/N with 0 <= R < N, N > 1")
        args.emulate = (r_, n_)
    args.emulate_rank = None
    default_workload = args.config is None and args.scaling == "weak" and args.tracers == 1 and \
        args.mesh == "structured" and not (args.permuted or args.parity_levels or args.graph or args.transfers) and \
        args.vlimit == 1 and args.fct_iter == 1 and args.path == "split" and args.exchange == "rccl" and \
        not getattr(args, "emulate", None)
    if args.config is None:
        args.config = "1.2M x 80" if args.scaling == "weak" else "9.6M x 80"
    args.leg = "headline"

    ctx = Ctx()
    ctx.world = world = int(os.environ.get("WORLD_SIZE", "1"))
    ctx.rank = rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
    ctx.watchdog = Watchdog(rank)

    # worker pool and the all-cores CPU baseline first: their processes are spawned before this
    # process touches the GPU
    if args.check or (rank == 0 and world == 1 and not args.no_cpu_baseline):
        ctx.pool, ctx.nworkers = make_pool(world)
    cpu_all = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_all = cpu_per_gpu_share(args, ctx.pool, ctx.nworkers)
        log(f"cpu per-GPU share: {cpu_all}")

    # the stream probes (own processes, before this one touches the GPU): the headline's size (with
    # the 6-tracer batched pattern when the extra legs run) and the small partition's
    ceilings = {}
    extras_on = (default_workload and args.extras == "auto") or args.extras == "on"
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        ceilings[args.config] = stream_ceiling(args.config, 6 if extras_on else args.tracers)
        if extras_on and args.config != "127k x 47":
            ceilings["127k x 47"] = stream_ceiling("127k x 47")
        log(f"stream ceilings: {ceilings}")
    ceiling = ceilings.get(args.config)

    abi.dll()  # engine first: one HIP runtime for the process
    abi.set_mpi_rank(local_rank, world)  # reference set_mpi_rank_: device = rank % ndev
    if world > 1:
        import torch.distributed as dist
        # gloo reports its connections on stdout; the driver reads rank 0's one JSON line there, so
        # fd 1 goes to stderr while the group connects (for good on ranks other than 0)
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        ctx.watchdog.arm("gloo process group setup", args.comm_timeout)
        dist.init_process_group("gloo")
        dist.barrier()
        ctx.watchdog.disarm()
        sys.stdout.flush()
        if rank == 0:
            os.dup2(saved, 1)
        os.close(saved)
        ctx.dist = dist

    head = run_leg(args, ctx, headline=True, cpu_all=cpu_all, ceiling=ceiling)
    m, s = head["m"], head["s"]
    out = {
        "metric": METRIC, "value": head["value"], "unit": "cell-updates/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": head["ms_per_step"],
        "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (deterministic splitmix64 fields, periodic structured triangulation; no dataset)",
        "config": {"workload": workload_name(args, world, m),
                   "tracers": args.tracers, "vlimit": args.vlimit, "fct_iterations": args.fct_iter,
                   "nodes_per_gpu": m.N, "levels": m.L,
                   "global_nodes": global_dims(args, world)[0] * global_dims(args, world)[1],
                   "cells_per_gpu": s["cn"], "edge_cells_per_gpu": s["ce"],
                   "parallelism": (f"node partition y-strips x{world}, "
                                   + ("RCCL halo overlapped with interior phase 2" if args.exchange == "rccl"
                                      else "host/gloo halo (validation, not a benchmark)"))
                   if world > 1 else "1 GPU",
                   "path": args.path},
        "roofline": head["roofline"],
        "cpu_baseline": head["cpu"],
        "pass_roofline": head["pass_roofline"],
        "kernels": head["kernels"],
        "gpu_event_ms_per_step": head["gpu_event_ms_per_step"],
        "graph": bool(args.graph),
        "transfers": "reference transfer semantics, PCIe inside the timed step" if args.transfers else
                     "device resident (inputs in HBM before the timed region)",
        "setup_s": head["setup_s"],
        "pass_order": head["pass_order"],
        "plan": head.get("plan"),
    }
    if head["check"] is not None:
        out["check"] = head["check"]
    for k in ("ranks", "rccl_nranks", "rccl"):
        if k in head:
            out[k] = head[k]
    del head, m, s
    gc.collect()
    exact = out.get("check") is None or out["check"]["exact"]

    # ---- further BASELINE configs in the same run
    if extras_on:
        out["extra"] = {}

        def partial(stage):  # watchdog on rank 0: the headline is measured, print what there is
            if rank == 0:
                out["extra"]["error"] = f"watchdog: '{stage}' not done within its bound"
                print(json.dumps(out), flush=True)
        ctx.watchdog.on_fire = partial
        for name, over in select_legs(extra_legs(args, world), args.legs):
            la = copy.copy(args)
            for k, v in over.items():
                setattr(la, k, v)
            la.leg = name
            la.traffic = os.path.join(ROOT, "profiles", "none.json")  # the per-config traffic files below
            ctx.watchdog.arm(f"extra leg {name}", args.leg_timeout)
            t0 = time.perf_counter()
            # the 9.6M x 80 strip columns stream like 1.2M x 80's (same column shape, both far past the
            # caches): that probe is their ceiling
            lc = ceilings.get(la.config) or (ceilings.get("1.2M x 80") if la.config == "9.6M x 80" else None)
            try:
                rec = run_leg(la, ctx, ceiling=lc)
            except Exception as ex:  # an extra leg must not cost the measured headline its line
                ctx.watchdog.disarm()
                log(f"rank {rank}: extra leg {name} failed: {type(ex).__name__}: {ex}")
                out["extra"][name] = {"error": f"{type(ex).__name__}: {ex}"}
                exact = False
                if world > 1:
                    # the other ranks may wait in a collective of this leg: end the run here (their
                    # gloo calls fail once this rank is gone); rank 0 reports what was measured
                    if rank == 0:
                        print(json.dumps(out), flush=True)
                    sys.stderr.flush()
                    os._exit(4)
                continue
            ctx.watchdog.disarm()
            out["extra"][name] = compact(rec, la, world)
            out["extra"][name]["leg_s"] = round(time.perf_counter() - t0, 1)
            exact = exact and (rec["check"] is None or rec["check"]["exact"])
            del rec
            gc.collect()
            log(f"extra {name}: {out['extra'][name]['ms_per_step']} ms/step")
        ctx.watchdog.on_fire = None

    if rank == 0:
        print(json.dumps(out), flush=True)
    if ctx.dist is not None:
        ctx.dist.destroy_process_group()
    if ctx.pool is not None:
        ctx.pool.terminate()
    if not exact:
        sys.exit(1)  # a fast wrong answer is not a result


if __name__ == "__main__":
    main()
