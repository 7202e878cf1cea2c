"""CPU: node partition, halo lists and the multi-rank algorithm (gloo, world_size 2).

A partitioned pass (per rank: phase 1 on owned nodes, halo exchange of fct_plus/fct_minus, phase 2)
must reproduce the single-domain pass exactly on every owned node: local edges keep global order, so
every node's edge sums run in the same order (the property the GPU path relies on too).
"""
import os
import socket

import numpy as np
import pytest

from fesom2_amd import partition, synth

import oracle as O


def global_mesh(nx=32, ny=24, nl=11, seed=42):
    return synth.make_mesh(nx, ny, nl, seed=seed)


def parts_of(kind, g, nranks, nx=32, ny=24):
    if kind == "strips":
        return partition.strip_parts(nx, ny, nranks)
    rng = np.random.default_rng(5)
    return rng.integers(0, nranks, g.N).astype(np.int32)  # adversarial: scattered ownership


@pytest.mark.parametrize("kind", ["strips", "random"])
@pytest.mark.parametrize("nranks", [2, 3, 4])
def test_local_meshes_and_exchange_lists(kind, nranks):
    g = global_mesh()
    part = parts_of(kind, g, nranks)
    locs = [partition.local_mesh(g, part, r) for r in range(nranks)]
    assert sum(m.N for m, _ in locs) == g.N
    for r, (m, h) in enumerate(locs):
        NT = m.N + m.H
        assert m.elem2D_nodes.min() >= 1 and m.elem2D_nodes.max() <= NT
        assert m.edges.min() >= 1 and m.edges.max() <= NT
        assert m.edge_tri.max() <= m.T and (m.edge_tri.reshape(-1, 2)[:, 0] >= 1).all()
        assert (part[m.node_gid[: m.N]] == r).all() and (part[m.node_gid[m.N:]] != r).all()
        assert np.all(np.diff(m.edge_gid) > 0), "local edges must keep global order"
        for q in h.neighbors:
            # what r receives from q is exactly what q sends to r, in the same (global id) order
            mq, hq = locs[q]
            assert np.array_equal(m.node_gid[h.recv[q] - 1], mq.node_gid[hq.send[r] - 1])
        # every halo node is received from its owner
        got = np.concatenate([h.recv[q] for q in h.neighbors]) if h.neighbors else np.zeros(0, np.int32)
        assert np.array_equal(np.sort(got), np.arange(m.N + 1, NT + 1))


def partitioned_oracle_pass(g, part, nranks):
    """Phase 1 per rank -> exchange (direct copy by the lists) -> phase 2 per rank."""
    locs = [partition.local_mesh(g, part, r) for r in range(nranks)]
    fields = [synth.make_fields(m) for m, _ in locs]
    p1 = []
    for (m, _), f in zip(locs, fields):
        st, out = O.pre_comm(m, f)
        assert st == 5
        p1.append(out)
    L = g.L
    for r, (m, h) in enumerate(locs):
        for q in h.neighbors:
            src = locs[q][1].send[r] - 1
            dst = h.recv[q] - 1
            for k in ("plus", "minus"):
                p1[r][k].reshape(-1, L)[dst] = p1[q][k].reshape(-1, L)[src]
    outs = [O.post_comm(m, f, o["plus"], o["minus"]) for (m, _), f, o in zip(locs, fields, p1)]
    for o, q in zip(outs, p1):
        o.update(plus=q["plus"], minus=q["minus"])
    return locs, outs


@pytest.mark.parametrize("kind", ["strips", "random"])
@pytest.mark.parametrize("nranks", [2, 4])
def test_partitioned_pass_equals_single_domain(kind, nranks):
    g = global_mesh()
    want = O.full_pass(g, synth.make_fields(g))
    locs, outs = partitioned_oracle_pass(g, parts_of(kind, g, nranks), nranks)
    L = g.L
    for k in ("plus", "minus", "del_v", "del_h"):
        got = partition.gather_owned([m for m, _ in locs], lambda r: outs[r][k], L, g.N)
        assert np.array_equal(got, want[k]), k
    got = partition.gather_owned([m for m, _ in locs], lambda r: outs[r]["adf_v"], g.nl, g.N)
    assert np.array_equal(got, want["adf_v"])
    # every global edge is local to one or two ranks and limited identically on both
    adf_h = np.full((g.E, L), np.nan)
    for (m, _), o in zip(locs, outs):
        loc = o["adf_h"].reshape(-1, L)
        seen = ~np.isnan(adf_h[m.edge_gid])
        assert np.array_equal(adf_h[m.edge_gid][seen], loc[seen])
        adf_h[m.edge_gid] = loc
    assert np.array_equal(adf_h.reshape(-1), want["adf_h"])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _gloo_worker(rank, world, port, result_q):
    """One rank: oracle phase 1, halo exchange over gloo (packed buffers, like the RCCL path), phase 2."""
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = global_mesh()
        part = partition.strip_parts(32, 24, world)
        m, h = partition.local_mesh(g, part, rank)
        f = synth.make_fields(m)
        st, p1 = O.pre_comm(m, f)
        L = m.L
        plus, minus = p1["plus"].reshape(-1, L), p1["minus"].reshape(-1, L)
        reqs, recv_bufs = [], {}
        for q in h.neighbors:  # pack [node][plus | minus] like k_pack
            s = h.send[q] - 1
            buf = torch.from_numpy(np.concatenate([plus[s], minus[s]], axis=1).copy())
            reqs.append(dist.isend(buf, dst=q))
            rb = torch.empty((h.recv[q].size, 2 * L), dtype=torch.float64)
            recv_bufs[q] = rb
            reqs.append(dist.irecv(rb, src=q))
        for r in reqs:
            r.wait()
        for q in h.neighbors:  # unpack into the halo columns like k_unpack
            d = h.recv[q] - 1
            plus[d] = recv_bufs[q][:, :L].numpy()
            minus[d] = recv_bufs[q][:, L:].numpy()
        out = O.post_comm(m, f, p1["plus"], p1["minus"])
        owned = {k: out[k][: m.N * L].reshape(m.N, L) for k in ("del_v", "del_h")}
        owned["plus"] = plus[: m.N]
        result_q.put((rank, st, m.node_gid[: m.N].copy(), {k: v.copy() for k, v in owned.items()}))
    finally:
        dist.destroy_process_group()


def test_gloo_two_ranks_matches_single_domain():
    mp = pytest.importorskip("torch.multiprocessing")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = global_mesh()
    want = O.full_pass(g, synth.make_fields(g))
    L = g.L
    seen = np.zeros(g.N, bool)
    for rank, st, gid, owned in results:
        assert st == 5
        seen[gid] = True
        for k, v in owned.items():
            assert np.array_equal(v, want[k].reshape(-1, L)[gid]), (rank, k)
    assert seen.all()


@pytest.mark.parametrize("nx,ny,nl,world,full", [(8, 6, 7, 2, False), (16, 9, 9, 3, False), (24, 16, 11, 4, True),
                                                 (5, 7, 6, 7, False), (10, 4, 5, 1, False), (12, 10, 9, 5, False)])
def test_strip_local_mesh_equals_the_cut_of_the_global_mesh(nx, ny, nl, world, full):
    """partition.strip_local_mesh builds a rank's y-strip from closed formulas of the structured
    numbering (no global mesh: what a rank of the 9.6M-node bench and the parallel check workers use);
    every array, count and exchange list equals local_mesh's cut of synth.make_mesh."""
    g = synth.make_mesh(nx, ny, nl, full_depth=full)
    parts = partition.strip_parts(nx, ny, world)
    row_part = parts.reshape(ny, nx)[:, 0]
    for r in range(world):
        y0, y1 = partition.strip_rows(ny, world, r)
        a, ha = partition.local_mesh(g, parts, r)
        b, hb = partition.strip_local_mesh(nx, ny, nl, y0, y1, full_depth=full, row_part=row_part, rank=r)
        for f in ("nl", "N", "H", "T", "E", "dim"):
            assert getattr(a, f) == getattr(b, f), (f, r)
        for f in ("elem2D_nodes", "edges", "edge_tri", "nie_num", "nie", "nlev_elem", "nlev_nod", "node_gid",
                  "edge_gid"):
            x, y = getattr(a, f), getattr(b, f)
            assert x.dtype == y.dtype and np.array_equal(x, y), (f, r)
        assert ha.neighbors == hb.neighbors
        for q in ha.neighbors:
            assert np.array_equal(ha.send[q], hb.send[q]) and np.array_equal(ha.recv[q], hb.recv[q]), (r, q)
