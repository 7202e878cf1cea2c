"""Trace-driven LRU model of one XCD's L2 during phase 1 (p1v) for candidate processing orders.

Sequential model: the first 150k positions of an order (one XCD's share at 1.2M x 80) access the
cluster columns (ttf+LO, 1280 B), the edge columns (fct_adf_h, 640 B) and ~5.1 KB of single-use
streams per node; prints L2-miss bytes per node against the algorithmic bytes.  It ranks orders
(index < BFS-64 patches < wide-front strips); it does not model in-flight concurrency, so absolute
excess is below what PMC measures.  usage: python tools/l2sim.py
"""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fesom2-accelerate_amd"))
import numpy as np
from fesom2_amd import synth

nx, ny, nl = 1600, 750, 81
m = synth.make_mesh(nx, ny, nl, full_depth=True)
N = m.N
E = m.E
ed = m.edges.reshape(-1, 2) - 1
# node->edge CSR ascending edge
deg = np.bincount(ed.ravel(), minlength=N)
ptr = np.zeros(N + 1, np.int64); ptr[1:] = np.cumsum(deg)
order_e = np.argsort(np.concatenate([ed[:, 0], ed[:, 1]]), kind="stable")
eid = np.concatenate([np.arange(E), np.arange(E)])[order_e]
oth = np.concatenate([ed[:, 1], ed[:, 0]])[order_e]
# cluster: nodes of elements around n
en = m.elem2D_nodes.reshape(-1, 3) - 1
nie = m.nie.reshape(-1, m.dim) - 1
def cluster(n):
    s = set()
    for e in nie[n]:
        if e >= 0: s.update(en[e].tolist())
    return s

def bfs_patches(patch=64):
    seen = np.zeros(N, bool); order = []; cursor = 0
    ptrl = ptr.tolist(); othl = oth.tolist()
    while len(order) < N:
        while seen[cursor]: cursor += 1
        q = [cursor]; seen[cursor] = True; cur = []; h = 0
        while h < len(q) and len(cur) < patch:
            v = q[h]; h += 1; cur.append(v)
            for k in range(ptrl[v], ptrl[v+1]):
                w = othl[k]
                if not seen[w]: seen[w] = True; q.append(w)
        for v in q[len(cur):]: seen[v] = False
        order.extend(sorted(cur))
    return np.array(order)

def strips(w):
    i = np.arange(N) % nx; j = np.arange(N) // nx
    band = i // w
    return np.lexsort((i, j, band))

def simulate(order, cap=4 << 20, nodes=150000, stream=5100):
    lru = collections.OrderedDict(); tot = 0; miss = 0; alg = 0
    eids = eid.tolist(); ptrl = ptr.tolist()
    uniq = 0
    def acc(key, size):
        nonlocal tot, miss
        if key in lru:
            lru.move_to_end(key); return
        lru[key] = size; tot += size; miss += size
        while tot > cap:
            _, s = lru.popitem(last=False); tot -= s
    for n in order[:nodes].tolist():
        for c in cluster(n): acc(('c', c), 1280)
        for k in range(ptrl[n], ptrl[n+1]): acc(('e', eids[k]), 640)
        uniq += 1; acc(('s', uniq), stream)
    # algorithmic: each cluster column once, each edge once
    sel = order[:nodes]
    cl = set(); es = set()
    for n in sel.tolist():
        cl |= cluster(n)
        es.update(eids[ptrl[n]:ptrl[n+1]])
    alg = len(cl) * 1280 + len(es) * 640 + nodes * stream
    return miss / nodes, alg / nodes

t = time.time()
orders = {"index": np.arange(N), "bfs64": bfs_patches(64)}
for w in (32, 64, 128, 256):
    orders[f"strip{w}"] = strips(w)
print("orders built", time.time() - t, flush=True)
for k, o in orders.items():
    t = time.time()
    mi, al = simulate(o)
    print(f"{k:10s} miss/node {mi:8.0f} B  alg/node {al:8.0f}  excess {mi/al-1:6.3f}  ({time.time()-t:.1f}s)", flush=True)
print("--- capacity sensitivity")
for cap in (1 << 20, 2 << 20):
    for k in ("bfs64", "strip64", "strip128"):
        mi, al = simulate(orders[k], cap=cap)
        print(f"cap {cap>>20}MB {k:10s} excess {mi/al-1:6.3f}", flush=True)
