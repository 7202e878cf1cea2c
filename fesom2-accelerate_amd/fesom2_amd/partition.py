"""Node partition of a global mesh into per-rank local meshes with a one-ring halo.

FESOM2's own domain decomposition (done by the Fortran host; the reference library only sees its
``myDim_nod2D`` / ``eDim_nod2D`` counts, src/fesom2-accelerate.cu:266, and the exchange of
fct_plus/fct_minus between the phases, docs/refactoring.md:199-200) is restated here for the
benchmark and the multi-rank tests:

* owned nodes of rank r: ``part == r``, numbered first in global order (``myDim_nod2D``);
* halo nodes: the other nodes of every element that has an owned node, numbered after the owned
  ones in global order (``eDim_nod2D``);
* local elements: elements with at least one owned node (``myDim_elem2D``);
* local edges: edges with at least one owned endpoint (``myDim_edge2D``);
* exchange lists: rank r sends to q the owned nodes of r that lie on an element with a q-owned
  node, and receives from q its halo nodes owned by q -- both sorted by global id, so the two
  sides agree on the order without talking.
"""
from __future__ import annotations

import dataclasses

import numpy as np

from .synth import Mesh


@dataclasses.dataclass
class Halo:
    neighbors: list          # neighbour ranks
    send: dict               # rank -> 1-based local owned node numbers to send
    recv: dict               # rank -> 1-based local halo node numbers to receive into


def strip_parts(nx, ny, nparts):
    """y-strips of a structured nx x ny mesh (row-major nodes): rows split as evenly as possible."""
    rows = np.arange(ny)
    part_of_row = (rows * nparts) // ny
    return np.repeat(part_of_row, nx).astype(np.int32)


def local_mesh(g: Mesh, part: np.ndarray, rank: int):
    """The local mesh of ``rank`` and its halo exchange lists."""
    assert g.H == 0, "partition a single-domain mesh"
    en = g.elem2D_nodes.reshape(-1, 3) - 1
    ed = g.edges.reshape(-1, 2) - 1
    et = g.edge_tri.reshape(-1, 2) - 1
    owned = part == rank
    owned_ids = np.flatnonzero(owned)
    elem_local = owned[en].any(axis=1)
    elem_ids = np.flatnonzero(elem_local)
    touched = np.zeros(g.N, bool)
    touched[en[elem_local].reshape(-1)] = True
    halo_ids = np.flatnonzero(touched & ~owned)
    node_ids = np.concatenate([owned_ids, halo_ids])
    n2l = np.full(g.N, -1, np.int64)
    n2l[node_ids] = np.arange(node_ids.size)
    e2l = np.full(g.T, -1, np.int64)
    e2l[elem_ids] = np.arange(elem_ids.size)
    edge_local = owned[ed].any(axis=1)
    edge_ids = np.flatnonzero(edge_local)

    l_en = (n2l[en[elem_ids]] + 1).astype(np.int32)
    assert (l_en > 0).all()
    l_ed = (n2l[ed[edge_ids]] + 1).astype(np.int32)
    assert (l_ed > 0).all()
    t = et[edge_ids]
    l_et = np.where(t >= 0, e2l[np.maximum(t, 0)] + 1, 0).astype(np.int32)
    assert (l_et[:, 0] > 0).all() and ((t[:, 1] < 0) | (l_et[:, 1] > 0)).all()
    nie_g = g.nie.reshape(-1, g.dim)[owned_ids] - 1
    l_nie = np.where(nie_g >= 0, e2l[np.maximum(nie_g, 0)] + 1, 0).astype(np.int32)
    assert ((nie_g < 0) | (l_nie > 0)).all()

    m = Mesh(nl=g.nl, N=int(owned_ids.size), H=int(halo_ids.size), T=int(elem_ids.size), E=int(edge_ids.size),
             dim=g.dim, elem2D_nodes=np.ascontiguousarray(l_en.reshape(-1)),
             edges=np.ascontiguousarray(l_ed.reshape(-1)), edge_tri=np.ascontiguousarray(l_et.reshape(-1)),
             nie_num=np.ascontiguousarray(g.nie_num[owned_ids]), nie=np.ascontiguousarray(l_nie.reshape(-1)),
             nlev_elem=np.ascontiguousarray(g.nlev_elem[elem_ids]),
             nlev_nod=np.ascontiguousarray(g.nlev_nod[node_ids]),
             node_gid=g.node_gid[node_ids].astype(np.int64), edge_gid=g.edge_gid[edge_ids].astype(np.int64),
             name=f"{g.name}[rank {rank}]")

    # exchange lists
    epart = part[en]  # (T, 3)
    halo_part = part[halo_ids]
    neighbors = sorted(set(int(q) for q in np.unique(halo_part)))
    send, recv = {}, {}
    for q in neighbors:
        # halo nodes owned by q, in global order (halo_ids is sorted)
        recv[q] = (n2l[halo_ids[halo_part == q]] + 1).astype(np.int32)
        # owned nodes of this rank on elements that have a q-owned node
        mixed = (epart == q).any(axis=1) & (epart == rank).any(axis=1)
        cand = np.unique(en[mixed].reshape(-1))
        cand = cand[part[cand] == rank]
        send[q] = (n2l[cand] + 1).astype(np.int32)
    return m, Halo(neighbors=neighbors, send=send, recv=recv)


def gather_owned(parts, field_of, stride, n_global):
    """Assemble a global (stride, N) field from the owned columns of each local mesh.

    ``parts`` is a list of local meshes, ``field_of(rank)`` the local field array of that rank.
    """
    out = np.zeros(n_global * stride)
    for r, m in enumerate(parts):
        a = np.asarray(field_of(r))[: m.N * stride].reshape(m.N, stride)
        out.reshape(n_global, stride)[m.node_gid[: m.N]] = a
    return out


def strip_rows(ny, nparts, rank):
    """The rows [y0, y1) rank owns in :func:`strip_parts`' y-strip partition."""
    rows = np.flatnonzero((np.arange(ny) * nparts) // ny == rank)
    return (int(rows[0]), int(rows[-1]) + 1) if rows.size else (0, 0)


def strip_edge_index(nx, ny, y0, y1, gids):
    """0-based position in :func:`strip_local_mesh`'s (= :func:`local_mesh`'s) edge list of owned rows
    [y0, y1) of each global edge id in ``gids`` (edges with an owned endpoint; closed form of the
    structured numbering: row j < ny-1 holds 3 nx edges (horizontal, vertical, diagonal per column),
    the last row nx horizontal ones; the row above the strip contributes its vertical and diagonal
    edges only)."""
    g = np.asarray(gids, dtype=np.int64)
    last = g >= 3 * nx * (ny - 1)
    j = np.where(last, ny - 1, g // (3 * nx))
    r = g - 3 * nx * j
    i = np.where(last, r, r // 3)
    kind = np.where(last, 0, r % 3)
    first = 2 * nx if y0 > 0 else 0
    idx = np.where(j < y0, 2 * i + kind - 1, first + 3 * nx * (j - y0) + np.where(last, i, 3 * i + kind))
    if np.any((j < y0 - 1) | (j >= y1) | ((j == y0 - 1) & (kind == 0))):
        raise ValueError("strip_edge_index: an edge without an endpoint in the strip")
    return idx


def strip_local_mesh(nx, ny, nl, y0, y1, seed=42, full_depth=False, row_part=None, rank=0, name=""):
    """The local mesh of owned rows [y0, y1) of :func:`fesom2_amd.synth.make_mesh`'s nx x ny
    triangulation -- bit for bit what :func:`local_mesh` cuts from the global mesh, built from the
    strip alone (every connectivity array is a closed formula of the structured numbering, element
    levels come from the same hash: ``synth_elem_levels``), so a rank of a 9.6M-node run or a worker
    of bench.py's parallel check never builds the global mesh.  ``row_part`` (rank per row) gives the
    exchange lists too (else ``None`` is returned for them)."""
    from . import synth
    assert 0 <= y0 < y1 <= ny and nx >= 3 and ny >= 2
    i = np.arange(nx, dtype=np.int64)
    nid = lambda ii, j: j * nx + ii % nx
    own = np.arange(y0 * nx, y1 * nx, dtype=np.int64)
    halo_rows = ([y0 - 1] if y0 > 0 else []) + ([y1] if y1 < ny else [])
    halo = np.concatenate([j * nx + i for j in halo_rows]) if halo_rows else np.zeros(0, np.int64)
    node_gid = np.concatenate([own, halo])
    N, H = own.size, halo.size

    def n2l(g):  # global node id -> 0-based local (owned, then halo rows in global order)
        j = g // nx
        out = g - y0 * nx
        out = np.where(j < y0, N + (g - (y0 - 1) * nx), out)
        return np.where(j >= y1, N + (nx if y0 > 0 else 0) + (g - y1 * nx), out)

    # local elements: quad rows [jq0, jq1] (every element touching an owned row), contiguous ids
    jq0, jq1 = max(0, y0 - 1), min(y1 - 1, ny - 2)
    q = (np.arange(jq0, jq1 + 1, dtype=np.int64)[:, None] * nx + i[None, :]).reshape(-1)
    qi, qj = q % nx, q // nx
    lower = np.stack([nid(qi, qj), nid(qi + 1, qj), nid(qi + 1, qj + 1)], axis=1)
    upper = np.stack([nid(qi, qj), nid(qi + 1, qj + 1), nid(qi, qj + 1)], axis=1)
    egl = np.stack([lower, upper], axis=1).reshape(-1, 3)  # element 2q, 2q+1
    t_off = 2 * nx * jq0
    T = egl.shape[0]

    # element levels of quad rows [jq0 - 1, jq1 + 1] (node levels of the halo rows need them)
    lq0, lq1 = max(0, jq0 - 1), min(ny - 2, jq1 + 1)
    lev = np.empty(2 * nx * (lq1 - lq0 + 1), np.int32)
    synth._lib().synth_elem_levels(nl, seed, 1 if full_depth else 0, 2 * nx * lq0, lev.size, synth._p(lev))
    lev_of = lambda t: lev[t - 2 * nx * lq0]

    def adjacent(g):  # (n, 6) global elements around nodes g (-1: none), ascending
        ii, j = g % nx, g // nx
        cand = []
        for dj, di, up in ((-1, -1, 0), (-1, -1, 1), (-1, 0, 1), (0, 0, 0), (0, 0, 1), (0, -1, 0)):
            jq = j + dj
            ok = (jq >= 0) & (jq <= ny - 2)
            cand.append(np.where(ok, 2 * (jq * nx + (ii + di) % nx) + up, -1))
        c = np.stack(cand, axis=1)
        c = np.where(c < 0, np.iinfo(np.int64).max, c)
        c.sort(axis=1)
        return np.where(c == np.iinfo(np.int64).max, -1, c)

    adj = adjacent(node_gid)
    nlev_nod = np.where(adj >= 0, lev_of(np.maximum(adj, 2 * nx * lq0)), 0).max(axis=1).astype(np.int32)
    adj_own = adj[:N]
    nie_num = (adj_own >= 0).sum(axis=1).astype(np.int32)
    nie = np.where(adj_own >= 0, adj_own - t_off + 1, 0).astype(np.int32)

    # local edges in global order: row y0 - 1 contributes its vertical/diagonal edges, owned rows all
    eg, en, et = [], [], []
    for j in range(max(0, y0 - 1), y1):
        base = 3 * nx * j
        h = j >= y0
        v = j < ny - 1
        if j < ny - 1:
            kinds = ([0] if h else []) + [1, 2]
            ids = base + 3 * i[:, None] + np.array(kinds)[None, :]
        else:
            kinds = [0]
            ids = (base + i)[:, None]
        for col, kind in enumerate(kinds):
            if kind == 0:  # horizontal (i, j)-(i+1, j)
                a, b = nid(i, j), nid(i + 1, j)
                if v:
                    t1, t2 = 2 * (j * nx + i) + 1, (2 * ((j - 1) * nx + i) + 1 + 1) if j > 0 else np.zeros(nx, np.int64)
                else:
                    t1, t2 = 2 * ((j - 1) * nx + i) + 1 + 1, np.zeros(nx, np.int64)
            elif kind == 1:  # vertical (i, j)-(i, j+1)
                a, b = nid(i, j), nid(i, j + 1)
                t1, t2 = 2 * (j * nx + i) + 1 + 1, 2 * (j * nx + (i - 1) % nx) + 1
            else:  # diagonal (i, j)-(i+1, j+1)
                a, b = nid(i, j), nid(i + 1, j + 1)
                t1, t2 = 2 * (j * nx + i) + 1, 2 * (j * nx + i) + 1 + 1
            eg.append(ids[:, col])
            en.append(np.stack([a, b], axis=1))
            et.append(np.stack([np.broadcast_to(t1, (nx,)), np.broadcast_to(t2, (nx,))], axis=1))
    order = np.argsort(np.concatenate(eg), kind="stable")
    edge_gid = np.concatenate(eg)[order]
    ed = np.concatenate(en)[order]
    etg = np.concatenate(et)[order]
    l_ed = (n2l(ed) + 1).astype(np.int32)
    l_et = np.where(etg > 0, etg - t_off, 0).astype(np.int32)
    m = synth.Mesh(nl=nl, N=int(N), H=int(H), T=int(T), E=int(edge_gid.size), dim=6,
                   elem2D_nodes=np.ascontiguousarray((n2l(egl) + 1).astype(np.int32).reshape(-1)),
                   edges=np.ascontiguousarray(l_ed.reshape(-1)), edge_tri=np.ascontiguousarray(l_et.reshape(-1)),
                   nie_num=nie_num, nie=np.ascontiguousarray(nie.reshape(-1)),
                   nlev_elem=np.ascontiguousarray(lev_of(np.arange(t_off, t_off + T))),
                   nlev_nod=nlev_nod, node_gid=node_gid, edge_gid=edge_gid.astype(np.int64),
                   name=name or f"{nx}x{ny}x{nl - 1}[rows {y0}:{y1}]")
    if row_part is None:
        return m, None
    row_part = np.asarray(row_part)
    neighbors, send, recv = [], {}, {}
    hpos = N
    for j in halo_rows:
        q_ = int(row_part[j])
        neighbors.append(q_)
        recv[q_] = np.arange(hpos + 1, hpos + nx + 1, dtype=np.int32)
        hpos += nx
        srow = y0 if j < y0 else y1 - 1
        send[q_] = (srow - y0) * nx + np.arange(1, nx + 1, dtype=np.int32)
    order = sorted(range(len(neighbors)), key=lambda k: neighbors[k])
    return m, Halo(neighbors=[neighbors[k] for k in order], send=send, recv=recv)
