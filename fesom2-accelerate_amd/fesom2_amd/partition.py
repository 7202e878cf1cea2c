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
