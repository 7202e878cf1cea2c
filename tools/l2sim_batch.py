"""Trace-driven LRU model of one XCD's L2 during the batched p1v (6 tracers, tiles (column group,
tracer), tracer fastest) for candidate processing orders of the 1.2M x 80 structured mesh.

Each tile of a node reads its tracer's cluster columns (ttf + LO, 1280 B each), its tracer's edge
columns (fct_adf_h, 640 B) and ~2.6 KB of single-use per-tracer streams; the first tracer of a
node also the shared mesh fields (~2.6 KB: area_inv, area, hnode, hnode_new), later tracers hit
them.  Sequential (no in-flight concurrency), so it ranks orders; the PMC numbers are the measure.
Orders: 4096-node BFS patches in ascending order (single rows), the same in row pairs of 3 + 3
(the product's batched plan on a large partition), and row pairs inside strips of W nodes
(strip_order, FESOM2_BATCH_STRIP).  usage: python tools/l2sim_batch.py [nodes=100000]
"""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fesom2-accelerate_amd"))
import numpy as np  # noqa: E402

from fesom2_amd import synth  # noqa: E402

nx, ny, nl = 1600, 750, 81
NTR = 6
m = synth.make_mesh(nx, ny, nl, full_depth=True)
N, E = m.N, m.E
ed = m.edges.reshape(-1, 2) - 1
deg = np.bincount(ed.ravel(), minlength=N)
ptr = np.zeros(N + 1, np.int64)
ptr[1:] = np.cumsum(deg)
order_e = np.argsort(np.concatenate([ed[:, 0], ed[:, 1]]), kind="stable")
eid = np.concatenate([np.arange(E), np.arange(E)])[order_e]
oth = np.concatenate([ed[:, 1], ed[:, 0]])[order_e]
en = m.elem2D_nodes.reshape(-1, 3) - 1
nie = m.nie.reshape(-1, m.dim) - 1
ptrl, othl, eidl = ptr.tolist(), oth.tolist(), eid.tolist()


def cluster(n):
    s = set()
    for e in nie[n]:
        if e >= 0:
            s.update(en[e].tolist())
    return s


def patches(size=4096):
    seen = np.zeros(N, bool)
    out, cursor = [], 0
    done = 0
    while done < N:
        while seen[cursor]:
            cursor += 1
        q, h, cur = [cursor], 0, []
        seen[cursor] = True
        while h < len(q) and len(cur) < size:
            v = q[h]
            h += 1
            cur.append(v)
            for k in range(ptrl[v], ptrl[v + 1]):
                w = othl[k]
                if not seen[w]:
                    seen[w] = True
                    q.append(w)
        for v in q[len(cur):]:
            seen[v] = False
        out.append(sorted(cur))
        done += len(cur)
    return out


def runs_of(cur):
    runs, s0 = [], 0
    for i in range(1, len(cur) + 1):
        if i == len(cur) or cur[i] != cur[i - 1] + 1:
            runs.append(cur[s0:i])
            s0 = i
    return runs


def row_pairs(cur, G=6):
    """3 nodes of a row over the 3 below them (structured numbering: the node below is +nx)."""
    runs, out, r = runs_of(cur), [], 0
    while r < len(runs):
        a = runs[r]
        if r + 1 < len(runs) and len(a) >= G and len(runs[r + 1]) >= G:
            b = runs[r + 1]
            ia, ib = 0, b.index(a[0] + nx) if (a[0] + nx) in b else 0
            out.extend(b[:ib])
            while ia < len(a) or ib < len(b):
                out.extend(a[ia:ia + 3])
                out.extend(b[ib:ib + 3])
                ia, ib = ia + 3, ib + 3
            r += 2
        else:
            out.extend(a)
            r += 1
    return out


def strip(cur, W):
    return sorted(cur, key=lambda v: ((v % nx) // W, v // nx, v % nx))


def order_of(kind, W=0):
    out = []
    for p in PATCHES:
        if kind == "single":
            out.extend(p)
        elif kind == "pairs":
            out.extend(row_pairs(p))
        else:
            out.extend(row_pairs(strip(p, W)))
    return out


def simulate(order, nodes, cap=4 << 20, own=2600, shared=2600):
    lru = collections.OrderedDict()
    tot = miss = 0

    def acc(key, size):
        nonlocal tot, miss
        if key in lru:
            lru.move_to_end(key)
            return
        lru[key] = size
        tot += size
        miss += size
        while tot > cap:
            _, s = lru.popitem(last=False)
            tot -= s
    cl_cache = {}
    alg_cl, alg_e = set(), set()
    G = 6
    for g0 in range(0, nodes, G):
        grp = order[g0:g0 + G]
        for tr in range(NTR):
            for n in grp:
                cl = cl_cache.get(n)
                if cl is None:
                    cl = cl_cache[n] = cluster(n)
                for c in cl:
                    acc(("c", tr, c), 1280)
                    alg_cl.add(c)
                for k in range(ptrl[n], ptrl[n + 1]):
                    acc(("e", tr, eidl[k]), 640)
                    alg_e.add(eidl[k])
                acc(("s", tr, n), own)
                acc(("m", n), shared)
    alg = NTR * (len(alg_cl) * 1280 + len(alg_e) * 640 + nodes * own) + nodes * shared
    return miss / alg


nodes = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
t = time.time()
PATCHES = patches(4096)
print(f"patches built {time.time() - t:.1f}s", flush=True)
for kind, W in (("single", 0), ("pairs", 0), ("strip", 12), ("strip", 18), ("strip", 24), ("strip", 36)):
    t = time.time()
    o = order_of(kind, W)
    r = simulate(o, nodes)
    print(f"{kind}{W or ''}: L2-miss bytes / algorithmic {r:.3f} ({time.time() - t:.0f}s)", flush=True)
