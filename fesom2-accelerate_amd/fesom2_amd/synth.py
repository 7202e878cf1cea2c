"""Deterministic synthetic FESOM-like meshes and fields (ctypes over ``lib/libfesom2_synth.so``).

The reference carries no mesh; its tuning scripts use unseeded random connectivity
(e.g. ``kernels/fct_ale_b1_horizontal.py:119-123``).  Here a periodic-x structured triangulation
with FESOM's array conventions is generated in C (``csrc/synth.c``), and every field value is a
pure function of (seed, field, global index), so a partition regenerates exactly the bits of the
whole mesh.  Sizes follow SURVEY.md §8 (T ~ 2N, E ~ 3N, dim = 6).
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import os

import numpy as np

from ._paths import lib_path

_synth = None


def _lib():
    global _synth
    if _synth is None:
        path = lib_path("libfesom2_synth.so")
        _synth = C.CDLL(path)
        _synth.synth_mesh_build.restype = C.c_int
        _synth.synth_mesh_build.argtypes = [C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_int] + [C.c_void_p] * 7
        _synth.synth_fill.argtypes = [C.c_uint64, C.c_int, C.c_int, C.c_int64, C.c_int, C.c_void_p,
                                      C.c_double, C.c_double, C.c_void_p]
    return _synth


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


# configs of BASELINE.json / SURVEY.md §8(d): name -> (nx, ny, nl)
CONFIGS = {
    "tiny": (16, 8, 11),
    "8k x 20": (128, 64, 21),
    "127k x 47": (512, 248, 48),
    "1.2M x 80": (1600, 750, 81),
    "9.6M x 80": (3200, 3000, 81),
}

FIELD_IDS = dict(ttf=10, LO=11, adf_v=12, adf_h=13, area=14, hnode=15, hnode_new=16, del_v=17, del_h=18)


@dataclasses.dataclass
class Mesh:
    """One (local) mesh in the reference's argument convention.

    N = myDim_nod2D, H = eDim_nod2D, T = myDim_elem2D, E = myDim_edge2D, nl levels (L = nl-1).
    Connectivity is int32 and 1-based; node_gid / edge_gid map local to global ids (fields are
    keyed on global ids).
    """
    nl: int
    N: int
    H: int
    T: int
    E: int
    dim: int
    elem2D_nodes: np.ndarray
    edges: np.ndarray
    edge_tri: np.ndarray
    nie_num: np.ndarray
    nie: np.ndarray
    nlev_elem: np.ndarray
    nlev_nod: np.ndarray
    node_gid: np.ndarray
    edge_gid: np.ndarray
    name: str = ""

    @property
    def L(self):
        return self.nl - 1

    @property
    def cells(self):
        """Cn = sum over owned nodes of (nlevels_nod2D - 1): the wet cells of one pass."""
        return int(np.sum(self.nlev_nod[: self.N].astype(np.int64) - 1))

    @property
    def edge_cells(self):
        """Ce = sum over local edges of max(nl1, nl2)."""
        t = self.edge_tri.reshape(-1, 2)
        nl1 = self.nlev_elem[t[:, 0] - 1].astype(np.int64) - 1
        second = t[:, 1] > 0
        nl2 = np.where(second, self.nlev_elem[np.maximum(t[:, 1] - 1, 0)].astype(np.int64) - 1, 0)
        return int(np.sum(np.maximum(nl1, nl2)))


def make_mesh(nx, ny, nl, seed=42, full_depth=False, name=""):
    """Periodic-x structured triangulation with nx*ny nodes (single domain: H = 0)."""
    N, T, E = nx * ny, 2 * nx * (ny - 1), 3 * nx * (ny - 1) + nx
    en = np.zeros(3 * T, np.int32)
    ed = np.zeros(2 * E, np.int32)
    et = np.zeros(2 * E, np.int32)
    nn = np.zeros(N, np.int32)
    nie = np.zeros(6 * N, np.int32)
    le = np.zeros(T, np.int32)
    ln = np.zeros(N, np.int32)
    rc = _lib().synth_mesh_build(nx, ny, nl, seed, 1 if full_depth else 0, _p(en), _p(ed), _p(et),
                                 _p(nn), _p(nie), _p(le), _p(ln))
    if rc:
        raise ValueError(f"synth_mesh_build({nx}, {ny}, {nl}) rejected the sizes")
    return Mesh(nl=nl, N=N, H=0, T=T, E=E, dim=6, elem2D_nodes=en, edges=ed, edge_tri=et, nie_num=nn,
                nie=nie, nlev_elem=le, nlev_nod=ln, node_gid=np.arange(N, dtype=np.int64),
                edge_gid=np.arange(E, dtype=np.int64), name=name or f"{nx}x{ny}x{nl - 1}")


def hilbert_key(xy, bits=16):
    """Index along a Hilbert curve of order ``bits`` of points in the unit square (vectorised xy2d)."""
    n = 1 << bits
    x = np.minimum((xy[:, 0] * n).astype(np.int64), n - 1)
    y = np.minimum((xy[:, 1] * n).astype(np.int64), n - 1)
    d = np.zeros(len(xy), np.int64)
    s = n >> 1
    while s > 0:
        rx = ((x & s) > 0).astype(np.int64)
        ry = ((y & s) > 0).astype(np.int64)
        d += s * s * ((3 * rx) ^ ry)
        # rotate the quadrant so the sub-curve has the canonical orientation
        flip = (ry == 0) & (rx == 1)
        x = np.where(flip, n - 1 - x, x)
        y = np.where(flip, n - 1 - y, y)
        swap = ry == 0
        x, y = np.where(swap, y, x), np.where(swap, x, y)
        s >>= 1
    return d


def delaunay_mesh(npts, nl, seed=11, full_depth=False, name="", numbering="scipy"):
    """Unstructured variant: the Delaunay triangulation of ``npts`` random points in the unit square.

    Node degrees vary (3 .. ~12, unlike the structured mesh's 6), so clusters and edge lists overflow
    the 8 inline NodeRec entries.  Same array conventions as :func:`make_mesh` (1-based, ``edge_tri``
    second entry 0 on the boundary, element levels uniform in [3, nl] unless ``full_depth``, node
    levels = max over the adjacent elements).

    ``numbering="scipy"``: the points' random order (scattered numbering, the plan's Cuthill-McKee case).
    ``numbering="hilbert"``: nodes numbered along a Hilbert curve and elements by the curve index of their
    centroid -- the locality a FESOM2 mesh has after its partitioner's renumbering (same triangulation,
    same edges set).
    """
    from scipy.spatial import Delaunay

    rng = np.random.default_rng(seed)
    pts = rng.random((npts, 2))
    tri = Delaunay(pts).simplices.astype(np.int64)  # (T, 3), 0-based
    if numbering == "hilbert":
        new = np.empty(npts, np.int64)
        new[np.argsort(hilbert_key(pts), kind="stable")] = np.arange(npts)
        tri = new[tri]
        tri = tri[np.argsort(hilbert_key(pts[np.argsort(new)][tri].mean(axis=1)), kind="stable")]
    elif numbering != "scipy":
        raise ValueError(f"delaunay_mesh: unknown numbering {numbering!r}")
    T = len(tri)
    e = np.concatenate([tri[:, [0, 1]], tri[:, [1, 2]], tri[:, [2, 0]]])
    e.sort(axis=1)
    uniq, inv = np.unique(e[:, 0] * npts + e[:, 1], return_inverse=True)
    E = len(uniq)
    edges = np.stack([uniq // npts, uniq % npts], axis=1)
    tri_of = np.tile(np.arange(T), 3)
    order = np.argsort(inv, kind="stable")
    cnt = np.bincount(inv, minlength=E)
    start = np.concatenate([[0], np.cumsum(cnt)[:-1]])
    et = np.zeros((E, 2), np.int64)
    et[:, 0] = tri_of[order[start]] + 1
    two = cnt == 2
    et[two, 1] = tri_of[order[start[two] + 1]] + 1
    # nod_in_elem2D: the elements around each node, padded with 0
    flat = tri.reshape(-1)
    deg = np.bincount(flat, minlength=npts)
    dim = int(deg.max())
    o = np.argsort(flat, kind="stable")
    pos = np.arange(flat.size) - np.concatenate([[0], np.cumsum(deg)[:-1]])[flat[o]]
    nie = np.zeros((npts, dim), np.int64)
    nie[flat[o], pos] = o // 3 + 1
    le = np.full(T, nl, np.int64) if full_depth else rng.integers(3, nl + 1, T)
    ln = np.zeros(npts, np.int64)
    np.maximum.at(ln, tri.reshape(-1), np.repeat(le, 3))
    i32 = lambda a: np.ascontiguousarray(a, dtype=np.int32).reshape(-1)
    return Mesh(nl=nl, N=npts, H=0, T=T, E=E, dim=dim, elem2D_nodes=i32(tri + 1), edges=i32(edges + 1),
                edge_tri=i32(et), nie_num=i32(deg), nie=i32(nie), nlev_elem=i32(le), nlev_nod=i32(ln),
                node_gid=np.arange(npts, dtype=np.int64), edge_gid=np.arange(E, dtype=np.int64),
                name=name or f"delaunay{npts}x{nl - 1}" + ("+hilbert" if numbering == "hilbert" else ""))


def config_mesh(name, full_depth=False, seed=42):
    nx, ny, nl = CONFIGS[name]
    return make_mesh(nx, ny, nl, seed=seed, full_depth=full_depth, name=name)


def fill(seed, field, dist, ncols, stride, gid, a, b):
    out = np.empty(int(ncols) * int(stride), np.float64)
    g = None if gid is None else np.ascontiguousarray(gid, dtype=np.int64)
    _lib().synth_fill(seed, FIELD_IDS[field] if isinstance(field, str) else field, dist, int(ncols), int(stride),
                      None if g is None else _p(g), a, b, _p(out))
    return out


FIELDS = ("ttf", "LO", "adf_v", "adf_h", "area", "area_inv", "hnode", "hnode_new", "del_v", "del_h")


def make_field(m: Mesh, name, seed=43, area_scale=1.0, adf_scale=0.5):
    """One field of :func:`make_fields` (the same bits): bench.py regenerates the pristine inputs of
    its parity check field by field instead of keeping a second host copy of a 9.6M-node mesh."""
    NT, L, nl = m.N + m.H, m.L, m.nl
    g = m.node_gid
    if name in ("ttf", "LO", "del_v", "del_h"):
        return fill(seed, name, 1, NT, L, g, 0.0, 1.0)
    if name == "adf_v":
        adf_v = fill(seed, "adf_v", 1, NT, nl, g, 0.0, adf_scale).reshape(NT, nl)
        # the bottom flux is always zero (docs/refactoring.md:232)
        adf_v[np.arange(nl)[None, :] >= (m.nlev_nod[:, None] - 1)] = 0.0
        return adf_v.reshape(-1)
    if name == "adf_h":
        return fill(seed, "adf_h", 1, m.E, L, m.edge_gid, 0.0, adf_scale)
    if name == "area":
        return fill(seed, "area", 0, NT, nl, g, 0.5 * area_scale, 2.0 * area_scale)
    if name == "area_inv":
        return 1.0 / make_field(m, "area", seed, area_scale, adf_scale)
    if name in ("hnode", "hnode_new"):
        return fill(seed, name, 0, NT, L, g, 5.0, 50.0)
    raise KeyError(name)


def make_fields(m: Mesh, seed=43, area_scale=1.0, adf_scale=0.5):
    """All per-tracer and per-mesh fields of one pass, keyed on global ids.

    Scales keep the limiter active (ratios in b2 of order one) so b2/b3 are exercised.
    """
    f = {k: make_field(m, k, seed, area_scale, adf_scale) for k in FIELDS if k != "area_inv"}
    f["area_inv"] = 1.0 / f["area"]
    return {k: f[k] for k in FIELDS}


def make_tracer_fields(m: Mesh, ntracers, seed=43, **kw):
    """Fields of ``ntracers`` tracers (seeds 43+k); the mesh fields (area, area_inv,
    hnode, hnode_new) of every tracer are those of the first, as one ocean state shares them."""
    out = [make_fields(m, seed=seed + k, **kw) for k in range(ntracers)]
    for f in out[1:]:
        for name in ("area", "area_inv", "hnode", "hnode_new"):
            f[name] = out[0][name]
    return out


def permute_mesh(m: Mesh, seed=7):
    """Shuffle node, element and edge numbering (an 'unstructured' stress variant).

    Global ids travel with the entities, so fields generated from the result describe the same
    physical problem; only the memory order changes.
    """
    assert m.H == 0
    rng = np.random.default_rng(seed)
    pn = rng.permutation(m.N)  # new id of old node i is pn[i]
    pe = rng.permutation(m.T)
    pg = rng.permutation(m.E)
    inv_n, inv_e, inv_g = np.argsort(pn), np.argsort(pe), np.argsort(pg)
    mapn = lambda a: (pn[a - 1] + 1).astype(np.int32)
    en = mapn(m.elem2D_nodes.reshape(-1, 3))[inv_e].reshape(-1)
    ed = mapn(m.edges.reshape(-1, 2))[inv_g].reshape(-1)
    t = m.edge_tri.reshape(-1, 2)
    t2 = np.where(t > 0, pe[np.maximum(t - 1, 0)] + 1, 0).astype(np.int32)
    et = t2[inv_g].reshape(-1)
    nie = m.nie.reshape(-1, m.dim)
    nie2 = np.where(nie > 0, pe[np.maximum(nie - 1, 0)] + 1, 0).astype(np.int32)[inv_n].reshape(-1)
    return dataclasses.replace(
        m, elem2D_nodes=np.ascontiguousarray(en), edges=np.ascontiguousarray(ed),
        edge_tri=np.ascontiguousarray(et), nie_num=np.ascontiguousarray(m.nie_num[inv_n]),
        nie=np.ascontiguousarray(nie2), nlev_elem=np.ascontiguousarray(m.nlev_elem[inv_e]),
        nlev_nod=np.ascontiguousarray(m.nlev_nod[inv_n]), node_gid=np.ascontiguousarray(m.node_gid[inv_n]),
        edge_gid=np.ascontiguousarray(m.edge_gid[inv_g]), name=m.name + "+perm")
