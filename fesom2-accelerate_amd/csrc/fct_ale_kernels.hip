// fct_ale_kernels.hip -- HIP kernels of the FCT-ALE limiter for CDNA4 (gfx950, wave64).
//
// Two kernel families:
//   * stepwise  -- one kernel per reference step (a1, a2, a3(+vlimit 2/3), b1v, b1h, b2, b3v, b3h,
//                  cv, ch).  They materialise fct_ttf_max/min and UV_rhs exactly like the reference
//                  GPU path (src/fesom2-accelerate.cu:294-376) and exist for alg_state granularity.
//   * fused     -- the production path.  Phase 1 (a1..b2) is ONE node-centric kernel that never
//                  materialises fct_ttf_max/min or UV_rhs; phase 2 is the edge-centric b3h kernel
//                  followed by ONE node-centric kernel for b3v + cv + ch.
//
// Parity design: every edge->node accumulation (b1-horizontal, c-horizontal) is a GATHER over a
// node->edge CSR kept in ascending edge order, which is the order in which the reference's edge
// loops add into a node (reference.cpp:406-425, docs/refactoring.md:303-314).  The per-node sums
// are therefore the same sequence of IEEE additions as the reference -- no atomics, bit-for-bit
// reproducible.  max/min are written as std::max/std::min ternaries, and the library is compiled
// with -ffp-contract=off so no multiply-add is fused (the x86-64 reference has none).
//
// Mapping: stepwise kernels use one wave64 per node column (or element / edge) with lanes over
// levels; the fused kernels give each wave a group of whole columns flattened over its lanes (see
// "fused kernels").  4 waves per 256-thread workgroup, and an XCD-aware block swizzle so each XCD's
// L2 walks a contiguous range of the (spatially sorted) mesh: neighbouring columns gathered by the
// cluster/edge loops are then L2/Infinity-Cache hits rather than HBM re-reads.
#include "f2a_device.hpp"

namespace f2a {

// ============================================================================ stepwise kernels

// a1: reference.cpp:306-319.  nodes 0..n_nodes (owned + halo), z < nlevels_nod2D - 1.
__global__ __launch_bounds__(kBlock) void k_a1(int n_nodes, int L, const int *__restrict__ nlev,
                                               const real *__restrict__ LO,
                                               const real *__restrict__ ttf, real *__restrict__ tmax,
                                               real *__restrict__ tmin)
{
    const int n = wave_item();
    if (n >= n_nodes) return;
    const int lane = threadIdx.x & 63;
    const int Ln = nlev[n] - 1;
    const size_t b = (size_t)n * L;
    for (int z = lane; z < Ln; z += kWave) {
        const real lo = LO[b + z], t = ttf[b + z];
        tmax[b + z] = RMAX(lo, t);
        tmin[b + z] = RMIN(lo, t);
    }
}

// a2: reference.cpp:321-351.  UV_rhs(2, L, elem) written as one 16-byte (max, min) pair.
__global__ __launch_bounds__(kBlock) void k_a2(int n_elem, int L, const int *__restrict__ nlev_elem,
                                               const int *__restrict__ elem_nodes,
                                               const real *__restrict__ tmax,
                                               const real *__restrict__ tmin, double2 *__restrict__ UV,
                                               real big)
{
    const int e = wave_item();
    if (e >= n_elem) return;
    const int lane = threadIdx.x & 63;
    const int Le = nlev_elem[e] - 1;
    const size_t k0 = (size_t)(elem_nodes[3 * (size_t)e] - 1) * L;
    const size_t k1 = (size_t)(elem_nodes[3 * (size_t)e + 1] - 1) * L;
    const size_t k2 = (size_t)(elem_nodes[3 * (size_t)e + 2] - 1) * L;
    double2 *uv = UV + (size_t)e * L;
    for (int z = lane; z < L; z += kWave) {
        double2 v;
        if (z < Le) {
            v.x = RMAX(RMAX(tmax[k0 + z], tmax[k1 + z]), tmax[k2 + z]);
            v.y = RMIN(RMIN(tmin[k0 + z], tmin[k1 + z]), tmin[k2 + z]);
        } else {
            v.x = -big;
            v.y = big;
        }
        uv[z] = v;
    }
}

// a3: reference.cpp:353-392 (vlimit 1) and docs/refactoring.md:113-148 (vlimit 2/3).
// LDS per wave: tvert_max, tvert_min and (vlimit 2/3) the node's a1 column, 3*L doubles.
__global__ __launch_bounds__(kBlock) void k_a3(int n_owned, int L, int vlimit,
                                               const int *__restrict__ nlev,
                                               const int *__restrict__ nie,
                                               const int *__restrict__ nie_num, int dim,
                                               const double2 *__restrict__ UV,
                                               const real *__restrict__ LO, real *__restrict__ tmax,
                                               real *__restrict__ tmin)
{
    extern __shared__ real lds[];
    const int n = wave_item();
    if (n >= n_owned) return;
    const int lane = threadIdx.x & 63;
    real *vmax = lds + (threadIdx.x >> 6) * 3 * L;
    real *vmin = vmax + L;
    real *a1c = vmin + L;
    const int Ln = nlev[n] - 1;
    const int ne = nie_num[n];
    const int *el = nie + (size_t)n * dim;
    const size_t b = (size_t)n * L;
    for (int z = lane; z < Ln; z += kWave) {
        const double2 v0 = UV[(size_t)(el[0] - 1) * L + z];
        real mx = v0.x, mn = v0.y;
        for (int k = 1; k < ne; k++) {
            const double2 v = UV[(size_t)(el[k] - 1) * L + z];
            mx = RMAX(mx, v.x);
            mn = RMIN(mn, v.y);
        }
        vmax[z] = mx;
        vmin[z] = mn;
        if (vlimit != 1) a1c[z] = tmax[b + z];
    }
    wave_lds_sync();
    for (int z = lane; z < Ln; z += kWave) {
        real tm, tn;
        if (vlimit == 1) {
            if (z == 0 || z == Ln - 1) {
                tm = vmax[z];
                tn = vmin[z];
            } else {
                tm = RMAX(RMAX(vmax[z - 1], vmax[z]), vmax[z + 1]);
                tn = RMIN(RMIN(vmin[z - 1], vmin[z]), vmin[z + 1]);
            }
        } else {
            tm = vmax[z];
            tn = vmin[z];
            if (z >= 1 && z < Ln - 1) {
                const real hmx = RMAX(RMAX(a1c[z - 1], a1c[z]), a1c[z + 1]);
                const real hmn = RMIN(RMIN(a1c[z - 1], a1c[z]), a1c[z + 1]);  // Fortran :121/:141 as written
                if (vlimit == 2) {
                    tm = RMAX(tm, hmx);
                    tn = RMIN(tn, hmn);
                } else {
                    tm = RMIN(tm, hmx);
                    tn = RMAX(tn, hmn);
                }
            }
        }
        const real lo = LO[b + z];
        tmax[b + z] = tm - lo;
        tmin[b + z] = tn - lo;
    }
}

// b1-vertical: reference.cpp:393-399 (fct_adf_v stride nl).
__global__ __launch_bounds__(kBlock) void k_b1v(int n_owned, int L, const int *__restrict__ nlev,
                                                const real *__restrict__ adf_v,
                                                real *__restrict__ plus, real *__restrict__ minus)
{
    const int n = wave_item();
    if (n >= n_owned) return;
    const int lane = threadIdx.x & 63;
    const int Ln = nlev[n] - 1;
    const size_t b = (size_t)n * L, a = (size_t)n * (L + 1);
    for (int z = lane; z < Ln; z += kWave) {
        const real v0 = adf_v[a + z], v1 = adf_v[a + z + 1];
        plus[b + z] = RMAX(0., v0) + RMAX(0., -v1);
        minus[b + z] = RMIN(0., v0) + RMIN(0., -v1);
    }
}

// b1-horizontal as an ascending-edge gather per owned node: reference.cpp:406-425.
__global__ __launch_bounds__(kBlock) void k_b1h(MeshPlanDev mp, int L, const real *__restrict__ adf_h,
                                                real *__restrict__ plus, real *__restrict__ minus)
{
    const int n = wave_item();
    if (n >= mp.n_owned) return;
    const int lane = threadIdx.x & 63;
    const int e0 = mp.edge_ptr[n], e1 = mp.edge_ptr[n + 1];
    int lmax = 0;
    for (int k = e0; k < e1; k++) lmax = max(lmax, edge_lev(mp.edges[k].code));
    const size_t b = (size_t)n * L;
    for (int z = lane; z < lmax; z += kWave) {
        real p = plus[b + z], m = minus[b + z];
        for (int k = e0; k < e1; k++) {
            const EdgeRef er = mp.edges[k];
            if (z < edge_lev(er.code)) {
                const real h = adf_h[(size_t)er.edge * L + z];
                if (er.code & 1) {
                    p += RMAX(0., -h);
                    m += RMIN(0., -h);
                } else {
                    p += RMAX(0., h);
                    m += RMIN(0., h);
                }
            }
        }
        plus[b + z] = p;
        minus[b + z] = m;
    }
}

// b2: reference.cpp:426-437.
__global__ __launch_bounds__(kBlock) void k_b2(int n_owned, int L, const int *__restrict__ nlev,
                                               const real *__restrict__ area_inv,
                                               const real *__restrict__ tmax,
                                               const real *__restrict__ tmin, real *__restrict__ plus,
                                               real *__restrict__ minus, real dt, real eps)
{
    const int n = wave_item();
    if (n >= n_owned) return;
    const int lane = threadIdx.x & 63;
    const int Ln = nlev[n] - 1;
    const size_t b = (size_t)n * L, a = (size_t)n * (L + 1);
    for (int z = lane; z < Ln; z += kWave) {
        const real ai = area_inv[a + z];
        real flux = plus[b + z] * dt * ai + eps;
        plus[b + z] = RMIN(1., tmax[b + z] / flux);
        flux = minus[b + z] * dt * ai - eps;
        minus[b + z] = RMIN(1., tmin[b + z] / flux);
    }
}


// b3-vertical: docs/refactoring.md:204-233, levels 0..nlev-2 of fct_adf_v(nl, nodes).
__global__ __launch_bounds__(kBlock) void k_b3v(int n_owned, int L, const int *__restrict__ nlev,
                                                const real *__restrict__ plus,
                                                const real *__restrict__ minus,
                                                real *__restrict__ adf_v)
{
    const int n = wave_item();
    if (n >= n_owned) return;
    const int lane = threadIdx.x & 63;
    const int Ln = nlev[n] - 1;
    const size_t b = (size_t)n * L, a = (size_t)n * (L + 1);
    const int top = Ln > 1 ? Ln : 1;  // the Fortran always limits nz = 1
    for (int z = lane; z < top; z += kWave) {
        const real f = adf_v[a + z];
        const real pm = z ? plus[b + z - 1] : 0., mm = z ? minus[b + z - 1] : 0.;
        const real ae = b3v_factor(z, f, pm, mm, plus[b + z], minus[b + z]);
        adf_v[a + z] = ae * f;
    }
}


// b3-horizontal, one wave per edge (docs/refactoring.md:237-263).  `list` (optional) selects edges.
__global__ __launch_bounds__(kBlock) void k_b3h(const int *__restrict__ list, int count, int L,
                                                const int *__restrict__ nlev_elem,
                                                const int *__restrict__ edges,
                                                const int *__restrict__ edge_tri,
                                                const real *__restrict__ plus,
                                                const real *__restrict__ minus,
                                                real *__restrict__ adf_h)
{
    int i = wave_item();
    if (i >= count) return;
    const int e = list ? list[i] : i;
    const int lane = threadIdx.x & 63;
    const size_t n1 = (size_t)(edges[2 * (size_t)e] - 1) * L;
    const size_t n2 = (size_t)(edges[2 * (size_t)e + 1] - 1) * L;
    const int el2 = edge_tri[2 * (size_t)e + 1] - 1;
    const int nl1 = nlev_elem[edge_tri[2 * (size_t)e] - 1] - 1;
    const int nl2 = el2 >= 0 ? nlev_elem[el2] - 1 : 0;
    const int lev = RMAX(nl1, nl2);
    real *h = adf_h + (size_t)e * L;
    for (int z = lane; z < lev; z += kWave) {
        const real f = h[z];
        h[z] = b3h_factor(f, plus[n1 + z], minus[n1 + z], plus[n2 + z], minus[n2 + z]) * f;
    }
}

// c-vertical: docs/refactoring.md:295-300 in the order of kernels/fct_ale_c_vertical.cu:9-12.
__global__ __launch_bounds__(kBlock) void k_cv(int n_owned, int L, const int *__restrict__ nlev,
                                               const real *__restrict__ ttf,
                                               const real *__restrict__ hnode,
                                               const real *__restrict__ LO,
                                               const real *__restrict__ hnode_new,
                                               const real *__restrict__ adf_v,
                                               const real *__restrict__ area,
                                               real *__restrict__ del_v, real dt)
{
    const int n = wave_item();
    if (n >= n_owned) return;
    const int lane = threadIdx.x & 63;
    const int Ln = nlev[n] - 1;
    const size_t b = (size_t)n * L, a = (size_t)n * (L + 1);
    for (int z = lane; z < Ln; z += kWave) {
        real t = del_v[b + z] - ttf[b + z] * hnode[b + z];
        t = t + LO[b + z] * hnode_new[b + z];
        t = t + (adf_v[a + z] - adf_v[a + z + 1]) * (dt / area[a + z]);
        del_v[b + z] = t;
    }
}

// c-horizontal as an ascending-edge gather per owned node (docs/refactoring.md:302-314,
// kernels/fct_ale_c_horizontal.cu:22-26 order): del[n1] += adf*(dt/area[n1]); del[n2] -= ...
__global__ __launch_bounds__(kBlock) void k_ch(MeshPlanDev mp, int L, const real *__restrict__ adf_h,
                                               const real *__restrict__ area,
                                               real *__restrict__ del_h, real dt)
{
    const int n = wave_item();
    if (n >= mp.n_owned) return;
    const int lane = threadIdx.x & 63;
    const int e0 = mp.edge_ptr[n], e1 = mp.edge_ptr[n + 1];
    int lmax = 0;
    for (int k = e0; k < e1; k++) lmax = max(lmax, edge_lev(mp.edges[k].code));
    const size_t b = (size_t)n * L, a = (size_t)n * (L + 1);
    for (int z = lane; z < lmax; z += kWave) {
        const real dta = dt / area[a + z];
        real d = del_h[b + z];
        for (int k = e0; k < e1; k++) {
            const EdgeRef er = mp.edges[k];
            if (z < edge_lev(er.code)) {
                const real h = adf_h[(size_t)er.edge * L + z];
                d = (er.code & 1) ? d - h * dta : d + h * dta;
            }
        }
        del_h[b + z] = d;
    }
}

// ============================================================================ fused kernels
// (block shape, level pairs and the shared gather helpers: f2a_device.hpp)

// Phase 1: a1 + a2 + a3 + b1v + b1h + b2 for the block's G columns.  Before the barrier every
// thread issues all of its loads (cluster gathers for tvert, edge gathers for b1h, its own column);
// after it the vertical 3-point stencil of tvert is read from LDS and the limiter ratios stored.
//
// VERT: the vertical half of phase 2 follows in the same kernel (b3v + cv read only the node's own
// column, so they need no halo exchange): plus/minus go through LDS to the neighbouring level slots,
// fct_adf_v is limited from the raw values the thread already holds and written after the barriers
// (every raw fct_adf_v read of the block happened before the first one), and del_ttf_advvert is
// updated -- the arithmetic of k_p2, so results are identical.  OPT & 64: b3v only, no cv (the
// reference entry sequence's fct_ale_pre_comm_acc_ in the fast mode: it has no del_ttf_advvert,
// hnode, hnode_new or area; fct_ale_c_acc_ does cv).
template <int VLIMIT, int C, int RB, int EB, bool NT, bool VERT = false, int OPT = 0, bool ODD = false>
__device__ __forceinline__ void p1_body(MeshPlanDev &mp, const P1Args &a0, int G, float invS)
{
    extern __shared__ real lds[];  // tvert max | tvert min | NodeRec[G]
    // tiles are (column group, tracer), tracer fastest (group_tracer)
    const int L = a0.nl - 1, S = (L + C - 1) / C;  // ODD: pairs, the last slot holds one level
    const int t = threadIdx.x;
    int tr = 0;
    const int grp = group_tracer(a0.tr.n, tr, c_tracer_major & 1, (c_tile_rev | a0.tr.order) & 1);
    const int first = grp * G;
    const int ncol = min(G, a0.n_owned - first);
    // doubles in front of the records: tvert max | min, or (OPT & 1024) the larger of that and the
    // cluster union's LO | ttf images, which then share the region (tvert is written after the union
    // has been read)
    int R0 = 2 * G * L;
    if constexpr ((OPT & 1024) != 0) R0 = max(R0, 2 * mp.cu_max * 2 * S);
    // OPT & 16 (VERT): the block-internal edges (both endpoints among its columns) are limited here,
    // after b2, from the plus/minus in LDS.  Wave 0 stages their entries and slot offsets (one
    // per lane, exclusive scan of ceil(lev/C)) while the records load.
    int4 *ie_ent = reinterpret_cast<int4 *>(lds + R0 + G * (int)(sizeof(NodeRec) / sizeof(real)));
    int *ie_off = reinterpret_cast<int *>(ie_ent + kMaxInternal);  // [kMaxInternal + 1]: + total
    // OPT & 32: the entries go global -> LDS by DMA after the records barrier instead (no VGPRs, off
    // the records' critical path: the two dependent loads above delay the block's first barrier),
    // and wave 0 scans their slot counts after the first barrier (read after the third)
    int int_i0 = 0, int_n = 0;
    if constexpr (VERT && (OPT & 16) && (OPT & 32)) {
        const int blk = first / G;
        int_i0 = mp.int_ptr[blk];  // block-uniform: scalar loads, waited for at the records barrier
        int_n = mp.int_ptr[blk + 1] - int_i0;
    }
    if constexpr (VERT && (OPT & 16) && !(OPT & 32)) {
        if (t < kWave) {
            const int blk = first / G, i0 = mp.int_ptr[blk], n = mp.int_ptr[blk + 1] - i0;
            const int4 ent = t < n ? mp.int_edges[i0 + t] : make_int4(0, 0, 0, 0);
            const int sl = t < n ? (ent.w + C - 1) / C : 0;
            int incl = sl;
#pragma unroll
            for (int d = 1; d < kWave; d <<= 1) {
                const int v = __shfl_up(incl, d);
                if (t >= d) incl += v;
            }
            if (t < kMaxInternal) {
                ie_ent[t] = ent;
                ie_off[t] = incl - sl;
            }
            if (t == kWave - 1) ie_off[kMaxInternal] = incl;
        }
    }
    // VLIMIT 2/3: max(LO, ttf) of the own column, for the 3-point vertical bound after the barrier
    // (behind the records and the internal-edge staging: p1_lds_bytes)
    real *cmx = lds + R0 + G * (int)(sizeof(NodeRec) / sizeof(real)) +
                ((VERT && (OPT & 16)) ? (int)(p1_internal_lds_bytes() / sizeof(real)) : 0);
    // OPT & 256 (with OPT & 16; the product default on large partitions, MeshPlanDev::int_stash; the
    // tuning build's FESOM2_P1V_STASH forces it): the internal edges' raw flux, kept by the first
    // endpoint's b1h gather ([slot][level], behind every other region)
    real *stash = nullptr;
    if constexpr (VERT && (OPT & 16) && (OPT & 256))
        stash = cmx + (VLIMIT != 1 ? G * L : 0);
    // OPT & 512 (MeshPlanDev::cu_ptr): the block's cluster union -- node ids, then the LO | ttf images
    // of its columns (2S doubles each, 16-byte aligned, behind every other region: p1_union_lds_bytes)
    real *uLO = nullptr, *uTT = nullptr;
    int *u_node = nullptr;
    int nU = 0;
    if constexpr ((OPT & 512) != 0) {
        const size_t off = (size_t)(cmx - lds) + (VLIMIT != 1 ? (size_t)G * L : 0) +
                           (((OPT & 16) && (OPT & 256)) ? (size_t)mp.int_max * L : 0);
        if constexpr ((OPT & 1024) != 0) {  // the images in front (R0), the ids behind everything
            uLO = lds;
            u_node = reinterpret_cast<int *>(lds + off);
        } else {
            uLO = lds + (off + 1) / 2 * 2;
            u_node = reinterpret_cast<int *>(uLO + 2 * (size_t)mp.cu_max * 2 * S);
        }
        const int blk = first / G, c0 = mp.cu_ptr[blk];
        nU = mp.cu_ptr[blk + 1] - c0;
        uTT = uLO + (size_t)nU * 2 * S;
        if (t < nU) u_node[t] = mp.cu_node[c0 + t];  // (read after stage_records' barrier)
    }
    const NodeRec *recs = stage_records(mp.node_rec, first, ncol, lds + R0);
    if constexpr (VERT && (OPT & 16) && (OPT & 32)) {
        if (t < int_n)  // wave 0 (int_n <= kMaxInternal = kWave): lane t's entry lands at ie_ent[t]
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(mp.int_edges + int_i0 + t),
                (__attribute__((address_space(3))) void *)ie_ent, 16, 0, 0);
    }
    int j, u;
    slot_of(t, S, invS, j, u);
    const int z0 = C * u;
    const bool last1 = ODD && z0 + 1 == L;
    const bool col = j < ncol;
    P1Args a = a0;
    if (tr) {
        a.ttf += tr * a.tr.node;
        a.LO += tr * a.tr.node;
        a.plus += tr * a.tr.node;
        a.minus += tr * a.tr.node;
        a.adf_v += tr * a.tr.lev;
        a.adf_h += tr * a.tr.edge;
        if (VERT && !(OPT & 64)) a.del_v += tr * a.tr.node;
    }
    if constexpr ((OPT & 512) != 0) {
        // the union's LO and ttf columns global -> LDS, 16 B per lane: item f of [array][slot][pair]
        // lands at uLO + 2f, i.e. each wave's 64 items fill 1 KB of LDS (landed at the next barrier)
        const int per = nU * S, items = (c_ablate & 32) ? 0 : 2 * per;
        for (int f0 = (t >> 6) * kWave; f0 < items; f0 += (int)blockDim.x) {
            const int f = f0 + (t & (kWave - 1));
            if (f < items) {
                const int arr = f >= per ? 1 : 0, g = f - arr * per;
                const int sl = (int)(((float)g + 0.5f) * invS), pr = g - sl * S;
                const real *src = (arr ? a.ttf : a.LO) + (size_t)u_node[sl] * L + 2 * pr;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                                 (__attribute__((address_space(3))) void *)(uLO + 2 * f0), 16, 0, 0);
            }
        }
    }
    const NodeRec &rec = recs[j];
    NodeInfo ni{};
    if (col) ni = rec.info;
    const int Ln = ni.Ln;
    const int nw = col ? max(0, min(C, Ln - z0)) : 0;  // wet cells of this thread
    real vx[C], vn[C], p[C], m[C];
#pragma unroll
    for (int c = 0; c < C; c++) vx[c] = vn[c] = p[c] = m[c] = 0.;
    size_t b = 0, ab = 0;
    real lo[C], tt[C];  // own LO / ttf
#pragma unroll
    for (int c = 0; c < C; c++) lo[c] = tt[c] = 0.;
    real v[C + 1];  // raw fct_adf_v at z0 .. z0+C (b1v; the VERT tail limits them)
#pragma unroll
    for (int c = 0; c <= C; c++) v[c] = 0.;
    real ai[C];  // area_inv
#pragma unroll
    for (int c = 0; c < C; c++) ai[c] = 0.;
    if (nw > 0) {
        b = (size_t)ni.n * L + z0;
        ab = (size_t)ni.n * a.nl + z0;
        if constexpr ((OPT & 4) != 0 && C == 2) {
            const f2a_d2u t = *reinterpret_cast<const f2a_d2u *>(a.adf_v + ab);  // one 16-B load at 8-B alignment
            v[0] = t.x;
            v[1] = t.y;
            v[2] = (nw == 2 && !(c_ablate & 8)) ? a.adf_v[ab + 2] : 0.;
        } else {
#pragma unroll
        for (int c = 0; c <= C; c++) v[c] = (c == 0 || c < nw + 1) ? ld1_s<NT>(a.adf_v + ab + c) : 0.;
        }
#pragma unroll
        for (int c = 0; c < C; c++) {
            p[c] = RMAX(0., v[c]) + RMAX(0., -v[c + 1]);  // b1-vertical, reference.cpp:393-399
            m[c] = RMIN(0., v[c]) + RMIN(0., -v[c + 1]);
        }
        const int ablate = c_ablate;
        const int nr = (ablate & 1) ? 0 : ni.r1 - ni.r0, ne = (ablate & 2) ? 0 : ni.e1 - ni.e0;
#pragma unroll
        for (int c = 0; c < C; c++) {
            const bool dry = z0 + c >= ni.zdry;
            vx[c] = dry ? -a.big : -INFINITY;
            vn[c] = dry ? a.big : INFINITY;
        }
        if constexpr ((OPT & 512) == 0) {
        const size_t bl = b;  // (odd L: the last slot's pair reads one level past the column, ldo)
        ldo_pre<C, ODD>(a.LO + bl, lo, last1);  // the own column: cluster bound (self last in the ring), b2, cv
        ldo_pre<C, ODD>(a.ttf + bl, tt, last1);
#pragma unroll
        for (int c = 0; c < C; c++)
            if (nr > 0 && z0 + c < ni.self_lev) {
                vx[c] = RMAX(vx[c], RMAX(lo[c], tt[c]));
                vn[c] = RMIN(vn[c], RMIN(lo[c], tt[c]));
            }
        const int no = nr > 0 ? nr - 1 : 0;  // the other cluster nodes
        cluster_bound<C, RB, ODD>(rec.ring, 0, min(no, kRecRing), a.LO, a.ttf, z0, L, vx, vn, last1);
        if (no > kRecRing)
            cluster_bound<C, RB, ODD>(mp.p_ring, ni.r0 + kRecRing, ni.r0 + no, a.LO, a.ttf, z0, L, vx, vn, last1);
        }
        auto add = [&](int c, real h, int second) {
            if (second) {  // ascending edge order: the reference's sum order (reference.cpp:406-425)
                p[c] += RMAX(0., -h);
                m[c] += RMIN(0., -h);
            } else {
                p[c] += RMAX(0., h);
                m[c] += RMIN(0., h);
            }
        };
        for_edges<C, EB, ODD>(rec.edge, 0, min(ne, kRecEdge), a.adf_h, z0, L, add, last1, stash);
        if (ne > kRecEdge)
            for_edges<C, EB, ODD>(mp.p_edges, ni.e0 + kRecEdge, ni.e1, a.adf_h, z0, L, add, last1, stash);
    }
    if constexpr ((OPT & 512) != 0) {
        // the union landed: own LO/ttf from slot j, the cluster bound from the slots the ring entries
        // carry -- the same values combined in the same order as the gathers above
        __builtin_amdgcn_s_waitcnt(0);  // this wave's DMA writes done before the barrier publishes them
        __syncthreads();
        if (nw > 0) {
            const int S2 = 2 * S;
#pragma unroll
            for (int c = 0; c < C; c++) {
                lo[c] = uLO[j * S2 + z0 + c];
                tt[c] = uTT[j * S2 + z0 + c];
            }
            const int nr = (c_ablate & 1) ? 0 : ni.r1 - ni.r0;
#pragma unroll
            for (int c = 0; c < C; c++)
                if (nr > 0 && z0 + c < ni.self_lev) {
                    vx[c] = RMAX(vx[c], RMAX(lo[c], tt[c]));
                    vn[c] = RMIN(vn[c], RMIN(lo[c], tt[c]));
                }
            const int no = nr > 0 ? nr - 1 : 0;
            for (int r = 0; r < no; r++) {
                const RingRef rr = r < kRecRing ? rec.ring[r] : mp.p_ring[ni.r0 + r];
                const int lv = rr.lev & kLevMask, sl = (rr.lev >> kStashShift) - 1;
                if (z0 >= lv) continue;
                real l2[C], t2[C];
                if (sl >= 0) {
#pragma unroll
                    for (int c = 0; c < C; c++) {
                        l2[c] = uLO[sl * S2 + z0 + c];
                        t2[c] = uTT[sl * S2 + z0 + c];
                    }
                } else {  // past the union's cap (MeshPlanDev::cu_max): from memory
                    ldo_pre<C, ODD>(a.LO + (size_t)rr.node * L + z0, l2, last1);
                    ldo_pre<C, ODD>(a.ttf + (size_t)rr.node * L + z0, t2, last1);
                }
#pragma unroll
                for (int c = 0; c < C; c++)
                    if (z0 + c < lv) {
                        vx[c] = RMAX(vx[c], RMAX(l2[c], t2[c]));
                        vn[c] = RMIN(vn[c], RMIN(l2[c], t2[c]));
                    }
            }
        }
        if constexpr ((OPT & 1024) != 0) __syncthreads();  // every union read done: tvert takes the region
    }
    real *tvx = lds, *tvn = lds + G * L;
    const int q = j * L + z0;
    if (col) {
#pragma unroll
        for (int c = 0; c < C; c++)
            if (!ODD || c == 0 || !last1) {  // ODD: the last slot's second level is the next column's
                tvx[q + c] = vx[c];
                tvn[q + c] = vn[c];
                if (VLIMIT != 1) cmx[q + c] = RMAX(lo[c], tt[c]);  // read on wet levels only
            }
    }
    __syncthreads();
    if constexpr (VERT && (OPT & 16) && (OPT & 32)) {
        if (t < kWave) {  // the DMA'd entries (landed: the barrier waited for vmcnt) -> slot offsets
            const int sl = t < int_n ? (ie_ent[t].w + C - 1) / C : 0;
            int incl = sl;
#pragma unroll
            for (int d = 1; d < kWave; d <<= 1) {
                const int v = __shfl_up(incl, d);
                if (t >= d) incl += v;
            }
            if (t < kMaxInternal) ie_off[t] = incl - sl;
            if (t == kWave - 1) ie_off[kMaxInternal] = incl;
        }
    }
    if (!VERT && nw == 0) return;
    real op[C], om[C];
#pragma unroll
    for (int c = 0; c < C; c++) op[c] = om[c] = 0.;
    if (nw > 0) {
    if constexpr ((OPT & 4) != 0) ld_nl<C, true>(a.area_inv + ab, nw, ai, 0.);
    else
#pragma unroll
    for (int c = 0; c < C; c++) ai[c] = c < nw ? ld1_s<NT>(a.area_inv + ab + c) : 0.;
#pragma unroll
    for (int c = 0; c < C; c++) {
        op[c] = om[c] = 0.;
        const int z = z0 + c;
        if (c >= nw) continue;
        real tm, tn;
        if (VLIMIT == 1) {
            if (z == 0 || z == Ln - 1) {
                tm = tvx[q + c];
                tn = tvn[q + c];
            } else {
                tm = RMAX(RMAX(tvx[q + c - 1], tvx[q + c]), tvx[q + c + 1]);
                tn = RMIN(RMIN(tvn[q + c - 1], tvn[q + c]), tvn[q + c + 1]);
            }
        } else {
            tm = tvx[q + c];
            tn = tvn[q + c];
            if (z >= 1 && z < Ln - 1) {  // levels z-1 .. z+1 of the own column, from LDS
                const real c0 = cmx[q + c - 1];
                const real c1 = cmx[q + c];
                const real c2 = cmx[q + c + 1];
                const real hmx = RMAX(RMAX(c0, c1), c2);
                const real hmn = RMIN(RMIN(c0, c1), c2);  // Fortran :121/:141 as written
                if (VLIMIT == 2) {
                    tm = RMAX(tm, hmx);
                    tn = RMIN(tn, hmn);
                } else {
                    tm = RMIN(tm, hmx);
                    tn = RMAX(tn, hmn);
                }
            }
        }
        real flux = p[c] * a.dt * ai[c] + a.eps;  // b2, reference.cpp:432-435
        op[c] = RMIN(1., (tm - lo[c]) / flux);
        flux = m[c] * a.dt * ai[c] - a.eps;
        om[c] = RMIN(1., (tn - lo[c]) / flux);
    }
    stv_s<C, NT>(a.plus + b, op, nw);
    stv_s<C, NT>(a.minus + b, om, nw);
    }
    if constexpr (VERT) {
        // ---- b3-vertical + c-vertical on the own column (as k_p2: docs/refactoring.md:204-233, :295-300)
        __syncthreads();  // the tvert stencil reads are done: the LDS takes plus/minus
        real *pl = lds, *mn = lds + G * L;
        if (col) {
#pragma unroll
            for (int c = 0; c < C; c++)
                if (!ODD || c == 0 || !last1) {
                    pl[q + c] = op[c];
                    mn[q + c] = om[c];
                }
        }
        __syncthreads();
        const int top = Ln > 1 ? Ln : 1;                   // the Fortran always limits nz = 1
        const int na = col ? max(0, min(C, top - z0)) : 0;  // cells whose fct_adf_v is limited
        if constexpr (OPT & 16) {
            // b3-horizontal of the block-internal edges (docs/refactoring.md:237-263): every raw read
            // of them (b1h of both endpoint columns) is behind the first barrier, no other block
            // touches them, and both endpoints' final plus/minus are in LDS
            const int total = ie_off[kMaxInternal];
            const int Sf = (L + C - 1) / C;  // slots of an edge that carries every level
            // (OPT & 32, entry count known) all edges full depth: the item's entry by division
            const bool uniform = (OPT & 32) && total == int_n * Sf;
            for (int w = t; w < total; w += (int)blockDim.x) {
                int lo_k = 0, hi_k = kMaxInternal - 1;  // last entry with ie_off <= w
                if (uniform) {
                    lo_k = w / Sf;
                } else {
                    while (lo_k < hi_k) {
                        const int mid = (lo_k + hi_k + 1) >> 1;
                        if (ie_off[mid] <= w) lo_k = mid;
                        else hi_k = mid - 1;
                    }
                }
                const int4 e = ie_ent[lo_k];
                const int zi = C * (w - ie_off[lo_k]);
                const bool l1 = ODD && zi + 1 == L;
                real f[C], out[C];
                const int nwi = min(C, e.w - zi);
                if constexpr ((OPT & 256) != 0) {
#pragma unroll
                    for (int c = 0; c < C; c++) f[c] = c < nwi ? stash[lo_k * L + zi + c] : 0.;
                } else {
                    ldo<C, ODD>(a.adf_h + (size_t)e.x * L + zi, f, l1);
                }
                const int q1 = e.y * L + zi, q2 = e.z * L + zi;
#pragma unroll
                for (int c = 0; c < C; c++)
                    out[c] = c < nwi ? b3h_factor(f[c], pl[q1 + c], mn[q1 + c], pl[q2 + c], mn[q2 + c]) * f[c] : 0.;
                stv_s<C, true>(const_cast<real *>(a.adf_h) + (size_t)e.x * L + zi, out, nwi);
            }
        }
        if (na <= 0) return;  // (the last statement with barriers is behind)
        if (nw == 0) {  // no wet cell (nlevels_nod2D <= 1): only nz = 1 is limited, from memory
            b = (size_t)ni.n * L + z0;
            ab = (size_t)ni.n * a.nl + z0;
#pragma unroll
            for (int c = 0; c <= C; c++) v[c] = c < 2 ? a.adf_v[ab + c] : 0.;
        }
        real pp[C + 2], mm[C + 2];  // plus/minus at z0-1 .. z0+C
        pp[0] = z0 ? pl[q - 1] : 0.;
        mm[0] = z0 ? mn[q - 1] : 0.;
#pragma unroll
        for (int c = 0; c < C; c++) {
            pp[c + 1] = c < nw ? op[c] : (c < na ? a.plus[b + c] : 0.);
            mm[c + 1] = c < nw ? om[c] : (c < na ? a.minus[b + c] : 0.);
        }
        const bool below = z0 + C < Ln;
        pp[C + 1] = below ? pl[q + C] : 0.;
        mm[C + 1] = below ? mn[q + C] : 0.;
        real lim[C + 1];
#pragma unroll
        for (int c = 0; c <= C; c++) {
            const int z = z0 + c;
            const bool lim_here = (c < C) ? (z < top) : (z < Ln);
            lim[c] = lim_here ? b3v_factor(z, v[c], pp[c], mm[c], pp[c + 1], mm[c + 1]) * v[c] : v[c];
        }
        real dv[C];
        if constexpr (OPT & 64) {
            (void)dv;
        } else if (nw > 0) {
            real del_v[C], hn[C], hnn[C], ar[C];
            if (c_ablate & 16) {
#pragma unroll
                for (int c = 0; c < C; c++) del_v[c] = hn[c] = hnn[c] = ar[c] = 1.;
            } else {
            ldo_s_pre<C, NT, ODD>(a.del_v + b, del_v, last1);
            ldo_s_pre<C, NT, ODD>(a.hnode + b, hn, last1);
            ldo_s_pre<C, NT, ODD>(a.hnode_new + b, hnn, last1);
            ld_nl<C, (OPT & 4) != 0>(a.area + ab, nw, ar, 1.);
            }
#pragma unroll
            for (int c = 0; c < C; c++) {
                const real dta = c < nw ? a.dt / ar[c] : 0.;
                real tv = del_v[c] - tt[c] * hn[c];  // kernels/fct_ale_c_vertical.cu:9-12 order
                tv = tv + lo[c] * hnn[c];
                dv[c] = tv + (lim[c] - lim[c + 1]) * dta;
            }
        }
#pragma unroll
        for (int c = 0; c < C; c++)
            if (!((OPT & 4) != 0 && C == 2 && na == 2) && c < na)
                st1_s<NT>(const_cast<real *>(a.adf_v) + ab + c, lim[c]);  // limited in place
        if constexpr ((OPT & 4) != 0 && C == 2)
            if (na == 2) {
                f2a_d2u t;
                t.x = lim[0];
                t.y = lim[1];
                *reinterpret_cast<f2a_d2u *>(const_cast<real *>(a.adf_v) + ab) = t;
            }
        if constexpr (!(OPT & 64))
            if (nw > 0) stv_s<C, NT>(a.del_v + b, dv, nw);
    }
}

template <int VLIMIT, int C, int RB, int EB, bool NT, bool VERT = false, int OPT = 0, bool ODD = false>
__global__ __launch_bounds__(1024) void k_p1(MeshPlanDev mp, P1Args a, int G, float invS)
{
    p1_body<VLIMIT, C, RB, EB, NT, VERT, OPT, ODD>(mp, a, G, invS);
}


// p1 held to W waves/SIMD (amdgpu_waves_per_eu): the register allocator trades a few spills for
// occupancy where a form sits just above a VGPR step (65 VGPRs = 7 waves, 74 = 6)
template <int W, int VLIMIT, int C, int RB, int EB, bool NT, bool VERT, int OPT, bool ODD = false>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(W))) void k_p1o(MeshPlanDev mp, P1Args a, int G,
                                                                                       float invS)
{
    p1_body<VLIMIT, C, RB, EB, NT, VERT, OPT, ODD>(mp, a, G, invS);
}


// Phase 2, horizontal half (after the exchange, with b3h): c-horizontal only (see k_p1 VERT).
template <int C, int KB, bool NT, bool PAIR = false, bool ODD = false>
__global__ __launch_bounds__(1024) void k_p2h(MeshPlanDev mp, P2Args a, int G, float invS)
{
    extern __shared__ real lds[];  // NodeRec[G]
    const int L = a.nl - 1, S = (L + C - 1) / C;
    int tr;
    const int first = group_tracer(a.tr.n, tr, c_tracer_major & 4, (c_tile_rev | a.tr.order) & 4) * G;
    if (tr) {
        a.del_h += tr * a.tr.node;
        a.adf_h += tr * a.tr.edge;
    }
    const int ncol = min(G, a.count - first);
    const NodeRec *recs = stage_records(a.nodes, first, ncol, lds);
    int j, u;
    slot_of(threadIdx.x, S, invS, j, u);
    const int z0 = C * u;
    const bool last1 = ODD && z0 + 1 == L;
    if (j >= ncol) return;
    const NodeInfo ni = recs[j].info;
    const int nw = max(0, min(C, ni.Ln - z0));
    if (nw <= 0) return;
    const size_t b = (size_t)ni.n * L + z0, ab = (size_t)ni.n * a.nl + z0;
    real dh[C], dta[C];
    ldo_s<C, NT, ODD>(a.del_h + b, dh, last1);
    if constexpr (PAIR && C == 2) {  // area: one 16-B load at 8-B alignment (ld_nl)
        const f2a_d2u t = NT ? __builtin_nontemporal_load(reinterpret_cast<const f2a_d2u *>(a.area + ab))
                             : *reinterpret_cast<const f2a_d2u *>(a.area + ab);
        dta[0] = a.dt / t.x;
        dta[1] = nw >= 2 ? a.dt / t.y : 0.;
    } else {
#pragma unroll
        for (int c = 0; c < C; c++) dta[c] = c < nw ? a.dt / ld1_s<NT>(a.area + ab + c) : 0.;
    }
    const int ne = ni.e1 - ni.e0;
    auto add = [&](int c, real h, int second) {
        dh[c] = second ? dh[c] - h * dta[c] : dh[c] + h * dta[c];  // docs/refactoring.md:311-312
    };
    for_edges<C, KB, ODD>(recs[j].edge, 0, min(ne, kRecEdge), a.adf_h, z0, L, add, last1);
    if (ne > kRecEdge) for_edges<C, KB, ODD>(mp.p_edges, ni.e0 + kRecEdge, ni.e1, a.adf_h, z0, L, add, last1);
    stv_s<C, NT>(a.del_h + b, dh, nw);
}


// Phase 2, edges: b3-horizontal (docs/refactoring.md:237-263) in place, G edge columns per block.
template <int C>
__global__ __launch_bounds__(1024) void k_b3h_g(const int4 *__restrict__ einfo, int n_edges, int L,
                                                int G, float invS, const real *__restrict__ plus,
                                                const real *__restrict__ minus,
                                                real *__restrict__ adf_h, Tracers trs)
{
    int j, u, tr;
    slot_of(threadIdx.x, L / C, invS, j, u);
    const int z0 = C * u;
    const int k = group_tracer(trs.n, tr, c_tracer_major & 2, c_tile_rev & 2) * G + j;
    plus += tr * trs.node;
    minus += tr * trs.node;
    adf_h += tr * trs.edge;
    if (j >= G || k >= n_edges) return;
    const int4 ei = einfo[k];  // {node1, node2, lev, edge}
    const int nw = min(C, ei.z - z0);
    if (nw <= 0) return;
    const size_t i = (size_t)ei.w * L + z0;
    const size_t i1 = (size_t)ei.x * L + z0, i2 = (size_t)ei.y * L + z0;
    real f[C], p1[C], m1[C], p2[C], m2[C], out[C];
    ldv<C>(adf_h + i, f);
    ldv<C>(plus + i1, p1);
    ldv<C>(minus + i1, m1);
    ldv<C>(plus + i2, p2);
    ldv<C>(minus + i2, m2);
#pragma unroll
    for (int c = 0; c < C; c++) out[c] = b3h_factor(f[c], p1[c], m1[c], p2[c], m2[c]) * f[c];
    stv<C>(adf_h + i, out, nw);
}


// b3-horizontal packed by depth: a block takes the consecutive edges of its descriptor, each with
// ceil(lev/2) level-pair slots (not L/2: shallow edges leave no idle slots), at most kB3hPackSlots
// slots, two per thread (both slots' loads in flight together, as k_b3h_u's two groups).  The
// block's edge infos and slot offsets go to LDS; a thread finds its edge by binary search.
// REG (reg = {P, s, first edge, edge count}): every edge of the list has s slots, so the greedy
// packing gave each block P = min(kB3hPackEdges, cap / s) consecutive edges (the last block fewer):
// a block computes its slice instead of loading a descriptor first, and drops the slot offsets.
template <bool NT, bool ODD, int H = 2, bool REG = false, bool STNT = NT>
__global__ __launch_bounds__(1024) void k_b3h_p(const int2 *__restrict__ desc, const unsigned short *__restrict__ off,
                                                const int4 *__restrict__ einfo, int L, const real *__restrict__ plus,
                                                const real *__restrict__ minus, real *__restrict__ adf_h, Tracers trs,
                                                int4 reg)
{
    __shared__ int4 s_ei[kB3hPackEdges];
    __shared__ int s_off[kB3hPackEdges + 1];
    int tr;
    const int g = group_tracer(trs.n, tr, c_tracer_major & 2, c_tile_rev & 2);
    plus += tr * trs.node;
    minus += tr * trs.node;
    adf_h += tr * trs.edge;
    const int t = threadIdx.x;
    int n, Sf;
    if constexpr (REG) {
        const int start = reg.z + g * reg.x;
        n = min(reg.x, reg.z + reg.w - start);
        Sf = reg.y;
        for (int i = t; i < n; i += blockDim.x) s_ei[i] = einfo[start + i];
    } else {
        const int2 dsc = desc[g];
        n = dsc.y;
        for (int i = t; i < n; i += blockDim.x) {
            const int4 ei = einfo[dsc.x + i];
            s_ei[i] = ei;
            s_off[i] = off[dsc.x + i];
            if (i == n - 1) s_off[n] = off[dsc.x + i] + (ei.z + 1) / 2;
        }
        // a block whose edges all carry every level (full depth: the common case) finds a slot's
        // edge by division; otherwise by binary search over the slot offsets
        Sf = (L + 1) / 2;
    }
    __syncthreads();
    constexpr int C = 2;
    int q[H], z0[H];
    bool act[H];
    real f[H][C], p1[H][C], m1[H][C], p2[H][C], m2[H][C];
    const int total = REG ? n * Sf : (n > 0 ? s_off[n] : 0);
    const bool uniform = REG || (n > 0 && total == n * Sf);
#pragma unroll
    for (int h = 0; h < H; h++) {
        const int slot = t + h * (int)blockDim.x;
        act[h] = n > 0 && slot < total;
        int lo = 0;
        if (uniform) {
            lo = min(slot / Sf, max(n - 1, 0));
        } else {
            int hi = n - 1;  // last edge with s_off <= slot
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (s_off[mid] <= slot) lo = mid;
                else hi = mid - 1;
            }
        }
        q[h] = lo;
        z0[h] = act[h] ? C * (slot - (uniform ? lo * Sf : s_off[lo])) : 0;
    }
#pragma unroll
    for (int h = 0; h < H; h++) {
        if (!act[h]) continue;
        const int4 ei = s_ei[q[h]];
        const bool last1 = ODD && z0[h] + 1 == L;
        ldo_s<C, NT, ODD>(adf_h + (size_t)ei.w * L + z0[h], f[h], last1);
        const size_t i1 = (size_t)ei.x * L + z0[h], i2 = (size_t)ei.y * L + z0[h];
        if (c_ablate & 64) {  // (timing only: no plus/minus gathers)
#pragma unroll
            for (int c = 0; c < C; c++) p1[h][c] = m1[h][c] = p2[h][c] = m2[h][c] = 0.5;
            continue;
        }
        ldo<C, ODD>(plus + i1, p1[h], last1);
        ldo<C, ODD>(minus + i1, m1[h], last1);
        ldo<C, ODD>(plus + i2, p2[h], last1);
        ldo<C, ODD>(minus + i2, m2[h], last1);
    }
#pragma unroll
    for (int h = 0; h < H; h++) {
        if (!act[h]) continue;
        const int4 ei = s_ei[q[h]];
        const int nw = min(C, ei.z - z0[h]);
        real out[C];
#pragma unroll
        for (int c = 0; c < C; c++) out[c] = b3h_factor(f[h][c], p1[h][c], m1[h][c], p2[h][c], m2[h][c]) * f[h][c];
        stv_s<C, STNT>(adf_h + (size_t)ei.w * L + z0[h], out, nw);  // !STNT: cache-allocating (pass_order)
    }
}

template <int C, int U, bool NT, bool ODD = false>
__global__ __launch_bounds__(1024) void k_b3h_u(const int4 *__restrict__ einfo, int n_edges, int L,
                                                int G, float invS, const real *__restrict__ plus,
                                                const real *__restrict__ minus,
                                                real *__restrict__ adf_h, Tracers trs)
{
    int tr;
    const int ug = group_tracer(trs.n, tr, c_tracer_major & 2, c_tile_rev & 2);
    b3h_groups<C, U, NT, ODD>(einfo, n_edges, L, G, invS, plus + tr * trs.node, minus + tr * trs.node,
                              adf_h + tr * trs.edge, ug);
}



// ============================================================================ reference-sequence
// entries on the fused path: fct_ale_inter_comm_acc_ (b3v) and fct_ale_c_acc_ (cv + ch) with the
// column-group shape of the production kernels (the one-wave-per-column kernels above stay for the
// stepwise path).

// b3-vertical, G consecutive owned columns per block (index order), level pairs.
template <int C, bool ODD>
__global__ __launch_bounds__(1024) void k_b3v_g(int n_owned, int L, int G, float invS, const int *__restrict__ nlev,
                                                const real *__restrict__ plus, const real *__restrict__ minus,
                                                real *__restrict__ adf_v)
{
    int j, u;
    slot_of(threadIdx.x, (L + C - 1) / C, invS, j, u);
    const int n = block_tile() * G + j;
    if (j >= G || n >= n_owned) return;
    const int z0 = C * u;
    const bool last1 = ODD && z0 + 1 == L;
    const int Ln = nlev[n] - 1;
    const int top = Ln > 1 ? Ln : 1;  // the Fortran always limits nz = 1
    const int na = min(C, top - z0);
    if (na <= 0) return;
    const size_t b = (size_t)n * L + z0, ab = (size_t)n * (L + 1) + z0;
    real f[C], p[C], m[C];
    ld_nl<C, true>(adf_v + ab, na, f, 0.);
    ldo<C, ODD>(plus + b, p, last1);
    ldo<C, ODD>(minus + b, m, last1);
    const real pm = z0 ? plus[b - 1] : 0., mm = z0 ? minus[b - 1] : 0.;
    real out[C];
#pragma unroll
    for (int c = 0; c < C; c++)
        out[c] = b3v_factor(z0 + c, f[c], c ? p[c - 1] : pm, c ? m[c - 1] : mm, p[c], m[c]) * f[c];
    if constexpr (C == 2) {
        if (na == 2) {
            f2a_d2u t;
            t.x = out[0];
            t.y = out[1];
            *reinterpret_cast<f2a_d2u *>(adf_v + ab) = t;
            return;
        }
    }
#pragma unroll
    for (int c = 0; c < C; c++)
        if (c < na) adf_v[ab + c] = out[c];
}

// c-step (docs/refactoring.md:292-314): c-vertical and c-horizontal of the block's G columns in
// processing order, one area load for both; the arithmetic of k_cv / k_p2h.
template <int C, int KB, bool ODD>
__global__ __launch_bounds__(1024) void k_c(MeshPlanDev mp, P2Args a, int G, float invS)
{
    static_assert(C == 2, "level pairs");
    extern __shared__ real lds[];  // NodeRec[G]
    const int L = a.nl - 1, S = (L + C - 1) / C;
    const int first = block_tile() * G;
    const int ncol = min(G, a.count - first);
    const NodeRec *recs = stage_records(a.nodes, first, ncol, lds);
    int j, u;
    slot_of(threadIdx.x, S, invS, j, u);
    const int z0 = C * u;
    const bool last1 = ODD && z0 + 1 == L;
    if (j >= ncol) return;
    const NodeInfo ni = recs[j].info;
    const int nw = max(0, min(C, ni.Ln - z0));
    if (nw <= 0) return;
    const size_t b = (size_t)ni.n * L + z0, ab = (size_t)ni.n * a.nl + z0;
    real dv[C], tt[C], hn[C], lo[C], hnn[C], dh[C], ar[C], v[C + 1], dta[C];
    ldo<C, ODD>(a.del_v + b, dv, last1);
    ldo<C, ODD>(a.ttf + b, tt, last1);
    ldo<C, ODD>(a.hnode + b, hn, last1);
    ldo<C, ODD>(a.LO + b, lo, last1);
    ldo<C, ODD>(a.hnode_new + b, hnn, last1);
    ldo<C, ODD>(a.del_h + b, dh, last1);
    ld_nl<C, true>(a.area + ab, nw, ar, 1.);
    {   // fct_adf_v at z0, z0+1 (a 16-byte load at 8-byte alignment, both inside the column: z0+1 <= L)
        // and z0+2 when both levels are wet (z0+2 <= Ln <= L)
        const f2a_d2u t = *reinterpret_cast<const f2a_d2u *>(a.adf_v + ab);
        v[0] = t.x;
        v[1] = t.y;
        v[2] = nw == 2 ? a.adf_v[ab + 2] : 0.;
    }
#pragma unroll
    for (int c = 0; c < C; c++) dta[c] = a.dt / ar[c];
#pragma unroll
    for (int c = 0; c < C; c++) {
        real t = dv[c] - tt[c] * hn[c];  // kernels/fct_ale_c_vertical.cu:9-12 order
        t = t + lo[c] * hnn[c];
        dv[c] = t + (v[c] - v[c + 1]) * dta[c];
    }
    const int ne = ni.e1 - ni.e0;
    auto add = [&](int c, real h, int second) {
        dh[c] = second ? dh[c] - h * dta[c] : dh[c] + h * dta[c];  // docs/refactoring.md:311-312
    };
    for_edges<C, KB, ODD>(recs[j].edge, 0, min(ne, kRecEdge), a.adf_h, z0, L, add, last1);
    if (ne > kRecEdge) for_edges<C, KB, ODD>(mp.p_edges, ni.e0 + kRecEdge, ni.e1, a.adf_h, z0, L, add, last1);
    stv<C>(a.del_v + b, dv, nw);
    stv<C>(a.del_h + b, dh, nw);
}

template <int C, int KB, bool NT>
__global__ __launch_bounds__(1024) void k_p2(MeshPlanDev mp, P2Args a, int G, float invS)
{
    extern __shared__ real lds[];  // NodeRec[G]
    int tr;
    const int first = group_tracer(a.tr.n, tr, c_tracer_major & 4, (c_tile_rev | a.tr.order) & 4) * G;
    if (tr) {
        a.plus += tr * a.tr.node;
        a.minus += tr * a.tr.node;
        a.ttf += tr * a.tr.node;
        a.LO += tr * a.tr.node;
        a.del_v += tr * a.tr.node;
        a.del_h += tr * a.tr.node;
        a.adf_v += tr * a.tr.lev;
        a.adf_h += tr * a.tr.edge;
    }
    const int ncol = min(G, a.count - first);
    const NodeRec *recs = stage_records(a.nodes, first, ncol, lds);
    p2_node_work<C, KB, NT>(mp, a, recs, ncol, invS);
}

// iter_yn phase 2, nodes (see P2IterArgs).  Every slot of a column also copies fct_adf_v2 into
// fct_adf_v for the levels the iteration does not assign (nz = 1, the bottom interface and the dry
// levels: the Fortran's whole-array `fct_adf_v = fct_adf_v2`); the last slot covers level nl-1.
template <int C>
__global__ __launch_bounds__(1024) void k_p2_iter(MeshPlanDev mp, P2IterArgs a, int G, float invS)
{
    extern __shared__ real lds[];  // NodeRec[G]
    const int L = a.nl - 1, S = L / C;
    const int t = threadIdx.x;
    int tr;
    const int first = group_tracer(a.tr.n, tr) * G;
    if (tr) {
        a.plus += tr * a.tr.node;
        a.minus += tr * a.tr.node;
        a.LO += tr * a.tr.node;
        a.adf_v += tr * a.tr.lev;
        a.adf_v2 += tr * a.tr.lev;
        a.adf_h += tr * a.tr.edge;
    }
    const int ncol = min(G, a.count - first);
    const NodeRec *recs = stage_records(a.nodes, first, ncol, lds);
    int j, u;
    slot_of(t, S, invS, j, u);
    const int z0 = C * u;
    const bool col = j < ncol;
    NodeInfo ni{};
    if (col) ni = recs[j].info;
    const int Ln = ni.Ln;
    const int top = Ln > 1 ? Ln : 1;
    const int na = col ? max(0, min(C, top - z0)) : 0;
    const int nw = col ? max(0, min(C, Ln - z0)) : 0;
    real rem[C], lo[C];
    const size_t b = (size_t)ni.n * L + z0, ab = (size_t)ni.n * a.nl + z0;
#pragma unroll
    for (int c = 0; c < C; c++) rem[c] = lo[c] = 0.;
    if (na > 0) {
        real pp[C + 2], mm[C + 2], f[C + 1];
        pp[0] = z0 ? a.plus[b - 1] : 0.;
        mm[0] = z0 ? a.minus[b - 1] : 0.;
        {
            real tp[C], tmn[C];
            ldv<C>(a.plus + b, tp);
            ldv<C>(a.minus + b, tmn);
#pragma unroll
            for (int c = 0; c < C; c++) {
                pp[c + 1] = tp[c];
                mm[c + 1] = tmn[c];
            }
        }
        const bool below = z0 + C < Ln;
        pp[C + 1] = below ? a.plus[b + C] : 0.;
        mm[C + 1] = below ? a.minus[b + C] : 0.;
#pragma unroll
        for (int c = 0; c <= C; c++) f[c] = a.adf_v[ab + c];
        real lim[C + 1];
#pragma unroll
        for (int c = 0; c <= C; c++) {
            const int z = z0 + c;
            const bool lim_here = (c < C) ? (z < top) : (z < Ln);
            const real ae = lim_here ? b3v_factor(z, f[c], pp[c], mm[c], pp[c + 1], mm[c + 1]) : 1.0;
            lim[c] = lim_here ? ae * f[c] : f[c];
            if (c < C) rem[c] = (1.0 - ae) * f[c];  // written for 1 <= z < Ln only
        }
        if (nw > 0) {
            real hnn[C], ar[C];
            ldv<C>(a.LO + b, lo);
            ldv<C>(a.hnode_new + b, hnn);
#pragma unroll
            for (int c = 0; c < C; c++) {
                ar[c] = c < nw ? a.area[ab + c] : 1.0;
                // LO + (adf_v(nz) - adf_v(nz+1)) * dt / area / hnode_new, left to right
                if (c < nw) lo[c] = lo[c] + (lim[c] - lim[c + 1]) * a.dt / ar[c] / hnn[c];
            }
            // the node's edges in ascending edge order (the Fortran edge loop's addition order), two
            // edges' raw flux and other-endpoint plus/minus in flight at a time, limited in-thread
            real pn[C], mn[C];
#pragma unroll
            for (int c = 0; c < C; c++) {
                pn[c] = pp[c + 1];
                mn[c] = mm[c + 1];
            }
            auto add = [&](int c, real lh, int second, int) {
                lo[c] = second ? lo[c] - lh * a.dt / ar[c] / hnn[c] : lo[c] + lh * a.dt / ar[c] / hnn[c];
            };
            const int ne = ni.e1 - ni.e0;
            for_edges_limited<C, 1>(recs[j].edge, 0, min(ne, kRecEdge), a.adf_h, a.plus, a.minus, pn, mn, z0, L, add);
            if (ne > kRecEdge)
                for_edges_limited<C, 1>(mp.p_edges, ni.e0 + kRecEdge, ni.e1, a.adf_h, a.plus, a.minus, pn, mn, z0, L,
                                        add);
        }
    }
    __syncthreads();  // every raw fct_adf_v read of the block precedes the writes
    if (!col) return;
    if (nw > 0) stv<C>(a.LO + b, lo, nw);
#pragma unroll
    for (int c = 0; c < C; c++) {
        const int z = z0 + c;
        if (z >= 1 && z < Ln) {
            a.adf_v2[ab + c] = rem[c];
            a.adf_v[ab + c] = rem[c];
        } else {
            a.adf_v[ab + c] = a.adf_v2[ab + c];
        }
    }
    if (z0 + C == L) a.adf_v[ab + C] = a.adf_v2[ab + C];  // level nl-1 (never wet)
}

// iter_yn phase 2, edges (after k_p2_iter has read the raw fluxes): fct_adf_h2 = (1-ae) adf_h on
// the edge's levels, then fct_adf_h <- fct_adf_h2 on every level.
template <int C>
__global__ __launch_bounds__(1024) void k_b3h_iter(const int4 *__restrict__ einfo, int n_edges, int L,
                                                   int G, float invS, const real *__restrict__ plus,
                                                   const real *__restrict__ minus,
                                                   real *__restrict__ adf_h, real *__restrict__ adf_h2,
                                                   Tracers trs)
{
    int j, u, tr;
    slot_of(threadIdx.x, L / C, invS, j, u);
    const int z0 = C * u;
    const int k = group_tracer(trs.n, tr, c_tracer_major & 2, c_tile_rev & 2) * G + j;
    if (j >= G || k >= n_edges) return;
    plus += tr * trs.node;
    minus += tr * trs.node;
    adf_h += tr * trs.edge;
    adf_h2 += tr * trs.edge;
    const int4 ei = einfo[k];
    const size_t i = (size_t)ei.w * L + z0;
    const size_t i1 = (size_t)ei.x * L + z0, i2 = (size_t)ei.y * L + z0;
    real f[C], h2[C], p1[C], m1[C], p2[C], m2[C];
    ldv_s<C, true>(adf_h + i, f);  // single-use streams: non-temporal
    // fct_adf_h2 keeps its old value (and fct_adf_h takes it) only on the levels below the edge's
    if (z0 + C > ei.z) ldv_s<C, true>(adf_h2 + i, h2);
    if (z0 < ei.z) {
        ldv<C>(plus + i1, p1);
        ldv<C>(minus + i1, m1);
        ldv<C>(plus + i2, p2);
        ldv<C>(minus + i2, m2);
    }
#pragma unroll
    for (int c = 0; c < C; c++)
        if (z0 + c < ei.z) h2[c] = (1.0 - b3h_factor(f[c], p1[c], m1[c], p2[c], m2[c])) * f[c];
    stv_s<C, true>(adf_h2 + i, h2, C);
    stv_s<C, true>(adf_h + i, h2, C);
}

// columns per block for S slots per column: G*S fills whole waves where possible (<= 1024 threads),
// times 2^shift (the plan's MeshPlanDev::gshift: shift < 0 halves the block; results do not depend
// on it)
int group_columns(int S, int shift)
{
    int best = 1;
    double best_waste = 1e30;
    for (int G = 1; G * S <= 1024; G *= 2) {
        const double waste = (double)(((G * S + kWave - 1) / kWave) * kWave) / (G * S);
        if (waste < best_waste - 1e-9) {
            best_waste = waste;
            best = G;
        }
        if (waste < 1.0 + 1e-9) break;
    }
    for (int k = 0; k < shift && best * 2 * S <= 1024; k++) best *= 2;
    for (int k = 0; k > shift && best > 1; k--) best /= 2;
    return best;
}


// levels per thread: 2 when columns are 16-byte aligned (L even), else 1

// ============================================================================ halo pack / unpack

// halo buffers: [list position][tracer][field a L | field b L] (field b optional)
__global__ __launch_bounds__(kBlock) void k_pack(const int *__restrict__ nodes, int count, int L,
                                                 int ntr, size_t stride,
                                                 const real *__restrict__ fa,
                                                 const real *__restrict__ fb,
                                                 real *__restrict__ buf)
{
    const int i = wave_item();  // list position * ntr + tracer
    if (i >= count * ntr) return;
    const int c = i / ntr, tr = i - c * ntr, nf = fb ? 2 : 1;
    const size_t src = tr * stride + (size_t)nodes[c] * L, dst = (size_t)i * nf * L;
    for (int z = threadIdx.x & 63; z < L; z += kWave) {
        buf[dst + z] = fa[src + z];
        if (fb) buf[dst + L + z] = fb[src + z];
    }
}

__global__ __launch_bounds__(kBlock) void k_unpack(const int *__restrict__ nodes, int count, int L,
                                                   int ntr, size_t stride,
                                                   const real *__restrict__ buf,
                                                   real *__restrict__ fa,
                                                   real *__restrict__ fb)
{
    const int i = wave_item();
    if (i >= count * ntr) return;
    const int c = i / ntr, tr = i - c * ntr, nf = fb ? 2 : 1;
    const size_t dst = tr * stride + (size_t)nodes[c] * L, src = (size_t)i * nf * L;
    for (int z = threadIdx.x & 63; z < L; z += kWave) {
        fa[dst + z] = buf[src + z];
        if (fb) fb[dst + z] = buf[src + L + z];
    }
}

// ============================================================================ launchers

#define F2A_LAUNCH(kernel, items, lds_bytes, s, ...)                                    \
    do {                                                                                \
        init_swizzle();                                                                 \
        if ((items) > 0)                                                                \
            hipLaunchKernelGGL(kernel, dim3(grid_for(items)), dim3(kBlock), (lds_bytes), \
                               (s), __VA_ARGS__);                                       \
        return hipGetLastError();                                                       \
    } while (0)

hipError_t launch_a1(int n_nodes, int nl, const int *nlev_nod, const real *LO, const real *ttf,
                     real *tmax, real *tmin, hipStream_t s)
{
    F2A_LAUNCH(k_a1, n_nodes, 0, s, n_nodes, nl - 1, nlev_nod, LO, ttf, tmax, tmin);
}

hipError_t launch_a2(int n_elem, int nl, const int *nlev_elem, const int *elem2D_nodes,
                     const real *tmax, const real *tmin, real *UV, real big, hipStream_t s)
{
    F2A_LAUNCH(k_a2, n_elem, 0, s, n_elem, nl - 1, nlev_elem, elem2D_nodes, tmax, tmin,
               reinterpret_cast<double2 *>(UV), big);
}

hipError_t launch_a3(int n_owned, int nl, int vlimit, const int *nlev_nod, const int *nie,
                     const int *nie_num, int dim, const real *UV, const real *LO, real *tmax,
                     real *tmin, hipStream_t s)
{
    const size_t lds = (size_t)kWavesPerBlock * 3 * (nl - 1) * sizeof(real);
    F2A_LAUNCH(k_a3, n_owned, lds, s, n_owned, nl - 1, vlimit, nlev_nod, nie, nie_num, dim,
               reinterpret_cast<const double2 *>(UV), LO, tmax, tmin);
}

hipError_t launch_b1v(int n_owned, int nl, const int *nlev_nod, const real *adf_v, real *plus,
                      real *minus, hipStream_t s)
{
    F2A_LAUNCH(k_b1v, n_owned, 0, s, n_owned, nl - 1, nlev_nod, adf_v, plus, minus);
}

hipError_t launch_b1h(const MeshPlanDev &mp, int nl, const real *adf_h, real *plus, real *minus,
                      hipStream_t s)
{
    F2A_LAUNCH(k_b1h, mp.n_owned, 0, s, mp, nl - 1, adf_h, plus, minus);
}

hipError_t launch_b2(int n_owned, int nl, const int *nlev_nod, const real *area_inv,
                     const real *tmax, const real *tmin, real *plus, real *minus, real dt,
                     real eps, hipStream_t s)
{
    F2A_LAUNCH(k_b2, n_owned, 0, s, n_owned, nl - 1, nlev_nod, area_inv, tmax, tmin, plus, minus,
               dt, eps);
}

hipError_t launch_b3v(int n_owned, int nl, const int *nlev_nod, const real *plus,
                      const real *minus, real *adf_v, hipStream_t s)
{
    F2A_LAUNCH(k_b3v, n_owned, 0, s, n_owned, nl - 1, nlev_nod, plus, minus, adf_v);
}

hipError_t launch_b3h(int n_edges, int nl, const int *nlev_elem, const int *edges,
                      const int *edge_tri, const real *plus, const real *minus, real *adf_h,
                      hipStream_t s)
{
    F2A_LAUNCH(k_b3h, n_edges, 0, s, (const int *)nullptr, n_edges, nl - 1, nlev_elem, edges,
               edge_tri, plus, minus, adf_h);
}

hipError_t launch_b3h_list(const int *edge_list, int count, int nl, const int *nlev_elem,
                           const int *edges, const int *edge_tri, const real *plus,
                           const real *minus, real *adf_h, hipStream_t s)
{
    F2A_LAUNCH(k_b3h, count, 0, s, edge_list, count, nl - 1, nlev_elem, edges, edge_tri, plus,
               minus, adf_h);
}

hipError_t launch_cv(int n_owned, int nl, const int *nlev_nod, const real *ttf, const real *hnode,
                     const real *LO, const real *hnode_new, const real *adf_v, const real *area,
                     real *del_v, real dt, hipStream_t s)
{
    F2A_LAUNCH(k_cv, n_owned, 0, s, n_owned, nl - 1, nlev_nod, ttf, hnode, LO, hnode_new, adf_v,
               area, del_v, dt);
}

hipError_t launch_ch(const MeshPlanDev &mp, int nl, const real *adf_h, const real *area,
                     real *del_h, real dt, hipStream_t s)
{
    F2A_LAUNCH(k_ch, mp.n_owned, 0, s, mp, nl - 1, adf_h, area, del_h, dt);
}

// L <= 1024 levels (one block per column at most); checked by the host entry points.


// The launchers below pick the production form of each kernel.  The forms that lost the A/B
// measurements of DESIGN.md §3 (other gather batches, load placements, cache policies, block
// shapes) are compiled into the tuning build only (F2A_TUNING, selected by FESOM2_* knobs there).

#if F2A_TUNING
template <int C, int RB, int EB>
static hipError_t p1_launch_tuning(const MeshPlanDev &mp, const P1Args &a, hipStream_t s, int G, int S, long groups)
{
    const float invS = 1.0f / (float)S;
    const size_t lds = p1_lds_bytes(G, a.nl - 1, a.vlimit, false);
    const bool NT = (knob("FESOM2_NT", 6) & 1) != 0;
    if constexpr (C == 2 && RB == 2 && EB == 2) {
        if (knob("FESOM2_NL_PAIR", 1)) {
            if (a.vlimit == 2) F2A_LAUNCH_GROUPS((k_p1<2, 2, 2, 2, false, false, 4>), groups, G, S, lds, s, mp, a, G, invS);
            if (a.vlimit == 3) F2A_LAUNCH_GROUPS((k_p1<3, 2, 2, 2, false, false, 4>), groups, G, S, lds, s, mp, a, G, invS);
            if (NT) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, false, 4>), groups, G, S, lds, s, mp, a, G, invS);
            F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, false, false, 4>), groups, G, S, lds, s, mp, a, G, invS);
        }
    }
    if (a.vlimit == 2) F2A_LAUNCH_GROUPS((k_p1<2, C, RB, EB, false>), groups, G, S, lds, s, mp, a, G, invS);
    if (a.vlimit == 3) F2A_LAUNCH_GROUPS((k_p1<3, C, RB, EB, false>), groups, G, S, lds, s, mp, a, G, invS);
    if (NT) F2A_LAUNCH_GROUPS((k_p1<1, C, RB, EB, true>), groups, G, S, lds, s, mp, a, G, invS);
    F2A_LAUNCH_GROUPS((k_p1<1, C, RB, EB, false>), groups, G, S, lds, s, mp, a, G, invS);
}
#endif

hipError_t launch_p1_fused(const MeshPlanDev &mp, const P1Args &a, hipStream_t s)
{
    if (odd_pairs(a.nl - 1) && a.vlimit == 1) {
        const int L = a.nl - 1, S = (L + 1) / 2, G = plan_columns(S, mp);
        const long groups = (long)(a.n_owned + G - 1) / G * a.tr.n;
        const size_t lds = 2 * (size_t)G * L * sizeof(real) + (size_t)G * sizeof(NodeRec);
        F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, false, false, 4, true>), groups, G, S, lds, s, mp, a, G, 1.0f / (float)S);
    }
    const int L = a.nl - 1, C = levels_per_thread(L), S = L / C, G = plan_columns(S, mp);
    const long groups = (long)(a.n_owned + G - 1) / G * a.tr.n;
#if F2A_TUNING
    // other gather batches (FESOM2_P1_BATCH = 10*RB + EB), cache policies
    switch (knob("FESOM2_P1_BATCH", 22)) {
    case 44: return C == 2 ? p1_launch_tuning<2, 4, 4>(mp, a, s, G, S, groups) : p1_launch_tuning<1, 4, 4>(mp, a, s, G, S, groups);
    case 24: return C == 2 ? p1_launch_tuning<2, 2, 4>(mp, a, s, G, S, groups) : p1_launch_tuning<1, 2, 4>(mp, a, s, G, S, groups);
    case 42: return C == 2 ? p1_launch_tuning<2, 4, 2>(mp, a, s, G, S, groups) : p1_launch_tuning<1, 4, 2>(mp, a, s, G, S, groups);
    case 88: return C == 2 ? p1_launch_tuning<2, 8, 8>(mp, a, s, G, S, groups) : p1_launch_tuning<1, 8, 8>(mp, a, s, G, S, groups);
    default: return C == 2 ? p1_launch_tuning<2, 2, 2>(mp, a, s, G, S, groups) : p1_launch_tuning<1, 2, 2>(mp, a, s, G, S, groups);
    }
#else
    // gathers in batches of 2 (58 VGPRs, 8 waves/SIMD), 16-byte pairs of the stride-nl arrays
    const float invS = 1.0f / (float)S;
    const size_t lds = p1_lds_bytes(G, L, a.vlimit, false);
    if (C == 2) {
        if (a.vlimit == 2) F2A_LAUNCH_GROUPS((k_p1<2, 2, 2, 2, false, false, 4>), groups, G, S, lds, s, mp, a, G, invS);
        if (a.vlimit == 3) F2A_LAUNCH_GROUPS((k_p1<3, 2, 2, 2, false, false, 4>), groups, G, S, lds, s, mp, a, G, invS);
        F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, false, false, 4>), groups, G, S, lds, s, mp, a, G, invS);
    }
    if (a.vlimit == 2) F2A_LAUNCH_GROUPS((k_p1<2, 1, 2, 2, false>), groups, G, S, lds, s, mp, a, G, invS);
    if (a.vlimit == 3) F2A_LAUNCH_GROUPS((k_p1<3, 1, 2, 2, false>), groups, G, S, lds, s, mp, a, G, invS);
    F2A_LAUNCH_GROUPS((k_p1<1, 1, 2, 2, false>), groups, G, S, lds, s, mp, a, G, invS);
#endif
}

int p1v_slots(int nl)
{
    const int L = nl - 1;
    return odd_pairs(L) ? (L + 1) / 2 : L / levels_per_thread(L);
}

int p1v_group_columns(int nl, int shift, int cols)
{
    if (cols > 0) return cols;
    const int L = nl - 1;
    if (odd_pairs(L)) return group_columns((L + 1) / 2, shift);
    return group_columns(L / levels_per_thread(L), shift);
}

// the launch_p1v forms with the internal-edge tail: the plan built the lists for this block size
bool p1v_limits_internal(const MeshPlanDev &mp, const P1Args &a)
{
    return mp.int_G > 0 && mp.int_ptr && mp.int_edges && a.vlimit >= 1 && a.vlimit <= 3 &&
           knob("FESOM2_P1V_B3H", 1) != 0 && p1v_group_columns(a.nl, mp.gshift, mp.gcols) == mp.int_G;
}


#if F2A_TUNING
// the measured forms of p1v (FESOM2_NT bit 2, FESOM2_NL_PAIR, FESOM2_P1V_INT_DMA)
static hipError_t launch_p1v_tuning(const MeshPlanDev &mp, const P1Args &a, hipStream_t s, bool in)
{
    const int L = a.nl - 1;
    if (odd_pairs(L) && a.vlimit != 1) {  // the product's forms (p1v_launch_G: pairs at every vlimit)
        const int S = (L + 1) / 2, G = plan_columns(S, mp);
        const long groups = (long)(a.n_owned + G - 1) / G * a.tr.n;
        const size_t lds = p1_lds_bytes(G, L, a.vlimit, in);
        const float inv = 1.0f / (float)S;
        if (a.vlimit == 2) {
            if (in) F2A_LAUNCH_GROUPS((k_p1<2, 2, 2, 2, true, true, 20, true>), groups, G, S, lds, s, mp, a, G, inv);
            F2A_LAUNCH_GROUPS((k_p1<2, 2, 2, 2, true, true, 4, true>), groups, G, S, lds, s, mp, a, G, inv);
        }
        if (in) F2A_LAUNCH_GROUPS((k_p1<3, 2, 2, 2, true, true, 20, true>), groups, G, S, lds, s, mp, a, G, inv);
        F2A_LAUNCH_GROUPS((k_p1<3, 2, 2, 2, true, true, 4, true>), groups, G, S, lds, s, mp, a, G, inv);
    }
    if (odd_pairs(L) && a.vlimit == 1) {
        const int S = (L + 1) / 2, G = plan_columns(S, mp);
        const long groups = (long)(a.n_owned + G - 1) / G * a.tr.n;
        const size_t lds = p1_lds_bytes(G, L, 1, in);
        const float inv = 1.0f / (float)S;
        if ((knob("FESOM2_NT", 6) & 4) != 0) {
            if (in && knob("FESOM2_P1V_INT_DMA", 1))
                F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 52, true>), groups, G, S, lds, s, mp, a, G, inv);
            if (in) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 20, true>), groups, G, S, lds, s, mp, a, G, inv);
            F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 4, true>), groups, G, S, lds, s, mp, a, G, inv);
        }
        if (in) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, false, true, 20, true>), groups, G, S, lds, s, mp, a, G, inv);
        F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, false, true, 4, true>), groups, G, S, lds, s, mp, a, G, inv);
    }
    const int C = levels_per_thread(L), S = L / C, G = plan_columns(S, mp);
    const long groups = (long)(a.n_owned + G - 1) / G * a.tr.n;
    const float invS = 1.0f / (float)S;
    const size_t lds = p1_lds_bytes(G, L, a.vlimit, in);
    // OPT bits of k_p1 (VERT): 4 16-B loads/stores of the stride-nl arrays (ld_nl, default), 16 the
    // block-internal edges' b3-horizontal, 32 their entries staged by DMA
    const int early = knob("FESOM2_NL_PAIR", 1) ? 4 : 0;
    const bool nt = (knob("FESOM2_NT", 6) & 4) != 0;
    if (a.vlimit != 1 && C == 2 && early == 4 && nt) {
        if (in && a.vlimit == 2) F2A_LAUNCH_GROUPS((k_p1<2, 2, 2, 2, true, true, 20>), groups, G, S, lds, s, mp, a, G, invS);
        if (in) F2A_LAUNCH_GROUPS((k_p1<3, 2, 2, 2, true, true, 20>), groups, G, S, lds, s, mp, a, G, invS);
        if (a.vlimit == 2) F2A_LAUNCH_GROUPS((k_p1<2, 2, 2, 2, true, true, 4>), groups, G, S, lds, s, mp, a, G, invS);
        F2A_LAUNCH_GROUPS((k_p1<3, 2, 2, 2, true, true, 4>), groups, G, S, lds, s, mp, a, G, invS);
    }
    if (in && a.vlimit == 2) {
        if (C == 2) F2A_LAUNCH_GROUPS((k_p1<2, 2, 2, 2, false, true, 16>), groups, G, S, lds, s, mp, a, G, invS);
        F2A_LAUNCH_GROUPS((k_p1<2, 1, 2, 2, false, true, 16>), groups, G, S, lds, s, mp, a, G, invS);
    }
    if (in && a.vlimit == 3) {
        if (C == 2) F2A_LAUNCH_GROUPS((k_p1<3, 2, 2, 2, false, true, 16>), groups, G, S, lds, s, mp, a, G, invS);
        F2A_LAUNCH_GROUPS((k_p1<3, 1, 2, 2, false, true, 16>), groups, G, S, lds, s, mp, a, G, invS);
    }
    if (in && C == 2 && early == 4 && nt && knob("FESOM2_P1V_INT_DMA", 1))
        F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 52>), groups, G, S, lds, s, mp, a, G, invS);
    if (in && C == 2 && early == 4 && nt)
        F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 20>), groups, G, S, lds, s, mp, a, G, invS);
    if (in && C == 2 && early == 4) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, false, true, 20>), groups, G, S, lds, s, mp, a, G, invS);
    if (in && C == 2) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, false, true, 16>), groups, G, S, lds, s, mp, a, G, invS);
    if (in) F2A_LAUNCH_GROUPS((k_p1<1, 1, 2, 2, false, true, 16>), groups, G, S, lds, s, mp, a, G, invS);
    if (C == 2) {
        if (a.vlimit == 2) F2A_LAUNCH_GROUPS((k_p1<2, 2, 2, 2, false, true>), groups, G, S, lds, s, mp, a, G, invS);
        if (a.vlimit == 3) F2A_LAUNCH_GROUPS((k_p1<3, 2, 2, 2, false, true>), groups, G, S, lds, s, mp, a, G, invS);
        if (early == 4 && nt) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 4>), groups, G, S, lds, s, mp, a, G, invS);
        if (early == 4) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, false, true, 4>), groups, G, S, lds, s, mp, a, G, invS);
        F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, false, true>), groups, G, S, lds, s, mp, a, G, invS);
    }
    if (a.vlimit == 2) F2A_LAUNCH_GROUPS((k_p1<2, 1, 2, 2, false, true>), groups, G, S, lds, s, mp, a, G, invS);
    if (a.vlimit == 3) F2A_LAUNCH_GROUPS((k_p1<3, 1, 2, 2, false, true>), groups, G, S, lds, s, mp, a, G, invS);
    F2A_LAUNCH_GROUPS((k_p1<1, 1, 2, 2, false, true>), groups, G, S, lds, s, mp, a, G, invS);
}
#endif

hipError_t launch_p1v(const MeshPlanDev &mp, const P1Args &a, hipStream_t s)
{
    if (!a.area || !a.hnode || !a.hnode_new || !a.del_v) return hipErrorInvalidValue;
    const bool in = p1v_limits_internal(mp, a);
#if F2A_TUNING
    // FESOM2_P1V_BATCH = 10*RB + EB: the production forms with other gather batches (cluster nodes /
    // edges per round trip; 22 = the product's)
    if (const int B = knob("FESOM2_P1V_BATCH", 22); B != 22 && a.vlimit == 1) {
        const int L = a.nl - 1;
        const bool odd = odd_pairs(L);
        if (odd || levels_per_thread(L) == 2) {
            const int S = (L + 1) / 2, G = plan_columns(S, mp);
            const long groups = (long)(a.n_owned + G - 1) / G * a.tr.n;
            const size_t lds = p1_lds_bytes(G, L, 1, in);
            const float inv = 1.0f / (float)S;
#define F2A_P1B(RB, EB)                                                                                                        \
            if (B == 10 * RB + EB) {                                                                                          \
                if (odd && in) F2A_LAUNCH_GROUPS((k_p1<1, 2, RB, EB, true, true, 52, true>), groups, G, S, lds, s, mp, a, G, inv); \
                if (odd) F2A_LAUNCH_GROUPS((k_p1<1, 2, RB, EB, true, true, 4, true>), groups, G, S, lds, s, mp, a, G, inv);      \
                if (in) F2A_LAUNCH_GROUPS((k_p1<1, 2, RB, EB, true, true, 52>), groups, G, S, lds, s, mp, a, G, inv);             \
                F2A_LAUNCH_GROUPS((k_p1<1, 2, RB, EB, true, true, 4>), groups, G, S, lds, s, mp, a, G, inv);                      \
            }
            F2A_P1B(3, 3)
            F2A_P1B(3, 2)
            F2A_P1B(2, 3)
            F2A_P1B(6, 2)
            F2A_P1B(2, 6)
#undef F2A_P1B
        }
    }
    // FESOM2_P1V_UNION = 1 (plan built with the cluster unions, MeshPlanDev::cu_ptr): the union's
    // LO/ttf columns staged into LDS once per block instead of each column's cluster gathers
    if (mp.cu_G > 0 && mp.cu_ptr && a.vlimit == 1) {
        const int L = a.nl - 1;
        const bool odd = odd_pairs(L);
        if (odd || levels_per_thread(L) == 2) {
            const int S = (L + 1) / 2, G = plan_columns(S, mp);
            if (G == mp.cu_G) {
                const long groups = (long)(a.n_owned + G - 1) / G * a.tr.n;
                const bool st = mp.int_stash && in;
                const size_t base = p1_lds_bytes(G, L, 1, in) + (st ? (size_t)mp.int_max * L * sizeof(real) : 0);
                const float inv = 1.0f / (float)S;
                if (knob("FESOM2_P1V_UNION", 2) != 1) {  // the union images share tvert's region (OPT 1024)
                    const size_t tv = 2 * (size_t)G * L * sizeof(real);
                    const size_t lds = std::max(tv, 2 * (size_t)mp.cu_max * 2 * S * sizeof(real)) + (base - tv) +
                                       (size_t)mp.cu_max * sizeof(int);
                    if (st && odd) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 52 | 256 | 1536, true>), groups, G, S, lds, s, mp, a, G, inv);
                    if (st) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 52 | 256 | 1536>), groups, G, S, lds, s, mp, a, G, inv);
                    if (in && odd) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 52 | 1536, true>), groups, G, S, lds, s, mp, a, G, inv);
                    if (in) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 52 | 1536>), groups, G, S, lds, s, mp, a, G, inv);
                    if (odd) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 4 | 1536, true>), groups, G, S, lds, s, mp, a, G, inv);
                    F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 4 | 1536>), groups, G, S, lds, s, mp, a, G, inv);
                }
                const size_t lds = p1_union_lds_bytes(base, mp.cu_max, S);
                if (st && odd) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 52 | 256 | 512, true>), groups, G, S, lds, s, mp, a, G, inv);
                if (st) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 52 | 256 | 512>), groups, G, S, lds, s, mp, a, G, inv);
                if (in && odd) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 52 | 512, true>), groups, G, S, lds, s, mp, a, G, inv);
                if (in) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 52 | 512>), groups, G, S, lds, s, mp, a, G, inv);
                if (odd) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 4 | 512, true>), groups, G, S, lds, s, mp, a, G, inv);
                F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 4 | 512>), groups, G, S, lds, s, mp, a, G, inv);
            }
        }
    }
    // FESOM2_P1V_STASH = 1 (plan built with the stash marks): the internal-edge forms keep the
    // internal edges' raw flux from b1h in LDS (int_max x L doubles more) instead of re-reading it
    if (mp.int_stash && in && a.vlimit == 1) {
        const int L = a.nl - 1;
        const bool odd = odd_pairs(L);
        if (odd || levels_per_thread(L) == 2) {
            const int S = (L + 1) / 2, G = plan_columns(S, mp);
            const long groups = (long)(a.n_owned + G - 1) / G * a.tr.n;
            const size_t lds = p1_lds_bytes(G, L, 1, in) + (size_t)mp.int_max * L * sizeof(real);
            const float inv = 1.0f / (float)S;
            if (knob("FESOM2_P1V_STASH", 1) == 2) {  // held to 8 waves/SIMD
                if (odd) F2A_LAUNCH_GROUPS((k_p1o<8, 1, 2, 2, 2, true, true, 52 | 256, true>), groups, G, S, lds, s, mp, a, G, inv);
                F2A_LAUNCH_GROUPS((k_p1o<8, 1, 2, 2, 2, true, true, 52 | 256>), groups, G, S, lds, s, mp, a, G, inv);
            }
            if (odd) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 52 | 256, true>), groups, G, S, lds, s, mp, a, G, inv);
            F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 52 | 256>), groups, G, S, lds, s, mp, a, G, inv);
        }
    }
    // FESOM2_P1V_WAVES = W: the production forms held to W waves/SIMD
    if (const int W = knob("FESOM2_P1V_WAVES", 0); W >= 6 && a.vlimit == 1) {
        const int L = a.nl - 1;
        const bool odd = odd_pairs(L);
        if (odd || levels_per_thread(L) == 2) {
            const int S = (L + 1) / 2, G = plan_columns(S, mp);
            const long groups = (long)(a.n_owned + G - 1) / G * a.tr.n;
            const size_t lds = p1_lds_bytes(G, L, 1, in);
            const float inv = 1.0f / (float)S;
#define F2A_P1O(WW)                                                                                                     \
            if (W == WW) {                                                                                            \
                if (odd && in) F2A_LAUNCH_GROUPS((k_p1o<WW, 1, 2, 2, 2, true, true, 52, true>), groups, G, S, lds, s, mp, a, G, inv); \
                if (odd) F2A_LAUNCH_GROUPS((k_p1o<WW, 1, 2, 2, 2, true, true, 4, true>), groups, G, S, lds, s, mp, a, G, inv);      \
                if (in) F2A_LAUNCH_GROUPS((k_p1o<WW, 1, 2, 2, 2, true, true, 52>), groups, G, S, lds, s, mp, a, G, inv);             \
                F2A_LAUNCH_GROUPS((k_p1o<WW, 1, 2, 2, 2, true, true, 4>), groups, G, S, lds, s, mp, a, G, inv);                      \
            }
            F2A_P1O(6)
            F2A_P1O(7)
            F2A_P1O(8)
#undef F2A_P1O
        }
    }
    return launch_p1v_tuning(mp, a, s, in);
#else
    const int L = a.nl - 1;
    // OPT 4: 16-byte loads/stores of the stride-nl arrays; +16 the block-internal edges'
    // b3-horizontal, +32 their entries staged into LDS by DMA, +256 their raw flux kept in LDS by
    // the b1h gather (plans with MeshPlanDev::int_stash: batched calls on large partitions), +512
    // the block's cluster union staged into LDS by DMA (plans with MeshPlanDev::cu_ptr: small
    // partitions), +1024 its images in tvert's region.  NT: the single-use streams (plus/minus/del_v
    // stores, the tail's del_v/hnode/hnode_new loads) non-temporal.
    if (mp.cu_G > 0 && mp.cu_ptr && a.vlimit == 1 && (odd_pairs(L) || levels_per_thread(L) == 2)) {
        const int S = (L + 1) / 2, G = plan_columns(S, mp);
        if (G == mp.cu_G) {
            const long groups = (long)(a.n_owned + G - 1) / G * a.tr.n;
            const bool st = mp.int_stash && in;
            const size_t base = p1_lds_bytes(G, L, 1, in) + (st ? (size_t)mp.int_max * L * sizeof(real) : 0);
            const size_t tv = 2 * (size_t)G * L * sizeof(real);
            const size_t lds = std::max(tv, 2 * (size_t)mp.cu_max * 2 * S * sizeof(real)) + (base - tv) +
                               (size_t)mp.cu_max * sizeof(int);
            const float inv = 1.0f / (float)S;
            if (st && odd_pairs(L)) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 52 | 256 | 1536, true>), groups, G, S, lds, s, mp, a, G, inv);
            if (st) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 52 | 256 | 1536>), groups, G, S, lds, s, mp, a, G, inv);
            if (in && odd_pairs(L)) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 52 | 1536, true>), groups, G, S, lds, s, mp, a, G, inv);
            if (in) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 52 | 1536>), groups, G, S, lds, s, mp, a, G, inv);
            if (odd_pairs(L)) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 4 | 1536, true>), groups, G, S, lds, s, mp, a, G, inv);
            F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 4 | 1536>), groups, G, S, lds, s, mp, a, G, inv);
        }
    }
    if (mp.int_stash && in && a.vlimit == 1 && (odd_pairs(L) || levels_per_thread(L) == 2)) {
        const int S = (L + 1) / 2, G = plan_columns(S, mp);
        const long groups = (long)(a.n_owned + G - 1) / G * a.tr.n;
        const size_t lds = p1_lds_bytes(G, L, 1, in) + (size_t)mp.int_max * L * sizeof(real);
        const float inv = 1.0f / (float)S;
        if (odd_pairs(L)) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 52 | 256, true>), groups, G, S, lds, s, mp, a, G, inv);
        F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 52 | 256>), groups, G, S, lds, s, mp, a, G, inv);
    }
    if (odd_pairs(L)) {  // odd L in level pairs, every vlimit (the 3-point bounds of vlimit 2/3 skip the pad level)
        const int S = (L + 1) / 2, G = plan_columns(S, mp);
        const long groups = (long)(a.n_owned + G - 1) / G * a.tr.n;
        const size_t lds = p1_lds_bytes(G, L, a.vlimit, in);
        const float inv = 1.0f / (float)S;
        switch (a.vlimit) {
        case 2:
            if (in) F2A_LAUNCH_GROUPS((k_p1<2, 2, 2, 2, true, true, 20, true>), groups, G, S, lds, s, mp, a, G, inv);
            F2A_LAUNCH_GROUPS((k_p1<2, 2, 2, 2, true, true, 4, true>), groups, G, S, lds, s, mp, a, G, inv);
        case 3:
            if (in) F2A_LAUNCH_GROUPS((k_p1<3, 2, 2, 2, true, true, 20, true>), groups, G, S, lds, s, mp, a, G, inv);
            F2A_LAUNCH_GROUPS((k_p1<3, 2, 2, 2, true, true, 4, true>), groups, G, S, lds, s, mp, a, G, inv);
        default:
            if (in) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 52, true>), groups, G, S, lds, s, mp, a, G, inv);
            F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 4, true>), groups, G, S, lds, s, mp, a, G, inv);
        }
    }
    const int C = levels_per_thread(L), S = L / C, G = plan_columns(S, mp);
    const long groups = (long)(a.n_owned + G - 1) / G * a.tr.n;
    const float invS = 1.0f / (float)S;
    const size_t lds = p1_lds_bytes(G, L, a.vlimit, in);
    if (C == 2) {
        switch (a.vlimit) {
        case 2:
            if (in) F2A_LAUNCH_GROUPS((k_p1<2, 2, 2, 2, true, true, 20>), groups, G, S, lds, s, mp, a, G, invS);
            F2A_LAUNCH_GROUPS((k_p1<2, 2, 2, 2, true, true, 4>), groups, G, S, lds, s, mp, a, G, invS);
        case 3:
            if (in) F2A_LAUNCH_GROUPS((k_p1<3, 2, 2, 2, true, true, 20>), groups, G, S, lds, s, mp, a, G, invS);
            F2A_LAUNCH_GROUPS((k_p1<3, 2, 2, 2, true, true, 4>), groups, G, S, lds, s, mp, a, G, invS);
        default:
            if (in) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 52>), groups, G, S, lds, s, mp, a, G, invS);
            F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 4>), groups, G, S, lds, s, mp, a, G, invS);
        }
    }
    // one level per thread (odd L at vlimit 2/3, or L < 3)
    switch (a.vlimit) {
    case 2:
        if (in) F2A_LAUNCH_GROUPS((k_p1<2, 1, 2, 2, false, true, 16>), groups, G, S, lds, s, mp, a, G, invS);
        F2A_LAUNCH_GROUPS((k_p1<2, 1, 2, 2, false, true>), groups, G, S, lds, s, mp, a, G, invS);
    case 3:
        if (in) F2A_LAUNCH_GROUPS((k_p1<3, 1, 2, 2, false, true, 16>), groups, G, S, lds, s, mp, a, G, invS);
        F2A_LAUNCH_GROUPS((k_p1<3, 1, 2, 2, false, true>), groups, G, S, lds, s, mp, a, G, invS);
    default:
        if (in) F2A_LAUNCH_GROUPS((k_p1<1, 1, 2, 2, false, true, 16>), groups, G, S, lds, s, mp, a, G, invS);
        F2A_LAUNCH_GROUPS((k_p1<1, 1, 2, 2, false, true>), groups, G, S, lds, s, mp, a, G, invS);
    }
#endif
}

// phase 1 + b3-vertical (+ the block-internal edges' b3-horizontal) without c-vertical: the
// reference sequence's fct_ale_pre_comm_acc_ in the fast mode (fesom2_set_path_(2))
hipError_t launch_p1_b3v(const MeshPlanDev &mp, const P1Args &a, hipStream_t s)
{
    const bool in = p1v_limits_internal(mp, a);
    const int L = a.nl - 1;
    if (odd_pairs(L)) {
        const int S = (L + 1) / 2, G = plan_columns(S, mp);
        const long groups = (long)(a.n_owned + G - 1) / G * a.tr.n;
        const size_t lds = p1_lds_bytes(G, L, a.vlimit, in);
        const float inv = 1.0f / (float)S;
        switch (a.vlimit) {
        case 2:
            if (in) F2A_LAUNCH_GROUPS((k_p1<2, 2, 2, 2, true, true, 20 | 64, true>), groups, G, S, lds, s, mp, a, G, inv);
            F2A_LAUNCH_GROUPS((k_p1<2, 2, 2, 2, true, true, 4 | 64, true>), groups, G, S, lds, s, mp, a, G, inv);
        case 3:
            if (in) F2A_LAUNCH_GROUPS((k_p1<3, 2, 2, 2, true, true, 20 | 64, true>), groups, G, S, lds, s, mp, a, G, inv);
            F2A_LAUNCH_GROUPS((k_p1<3, 2, 2, 2, true, true, 4 | 64, true>), groups, G, S, lds, s, mp, a, G, inv);
        default:
            if (in) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 52 | 64, true>), groups, G, S, lds, s, mp, a, G, inv);
            F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 4 | 64, true>), groups, G, S, lds, s, mp, a, G, inv);
        }
    }
    const int C = levels_per_thread(L), S = L / C, G = plan_columns(S, mp);
    const long groups = (long)(a.n_owned + G - 1) / G * a.tr.n;
    const float invS = 1.0f / (float)S;
    const size_t lds = p1_lds_bytes(G, L, a.vlimit, in);
    if (C == 2) {
        switch (a.vlimit) {
        case 2:
            if (in) F2A_LAUNCH_GROUPS((k_p1<2, 2, 2, 2, true, true, 20 | 64>), groups, G, S, lds, s, mp, a, G, invS);
            F2A_LAUNCH_GROUPS((k_p1<2, 2, 2, 2, true, true, 4 | 64>), groups, G, S, lds, s, mp, a, G, invS);
        case 3:
            if (in) F2A_LAUNCH_GROUPS((k_p1<3, 2, 2, 2, true, true, 20 | 64>), groups, G, S, lds, s, mp, a, G, invS);
            F2A_LAUNCH_GROUPS((k_p1<3, 2, 2, 2, true, true, 4 | 64>), groups, G, S, lds, s, mp, a, G, invS);
        default:
            if (in) F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 52 | 64>), groups, G, S, lds, s, mp, a, G, invS);
            F2A_LAUNCH_GROUPS((k_p1<1, 2, 2, 2, true, true, 4 | 64>), groups, G, S, lds, s, mp, a, G, invS);
        }
    }
    switch (a.vlimit) {
    case 2:
        if (in) F2A_LAUNCH_GROUPS((k_p1<2, 1, 2, 2, false, true, 16 | 64>), groups, G, S, lds, s, mp, a, G, invS);
        F2A_LAUNCH_GROUPS((k_p1<2, 1, 2, 2, false, true, 64>), groups, G, S, lds, s, mp, a, G, invS);
    case 3:
        if (in) F2A_LAUNCH_GROUPS((k_p1<3, 1, 2, 2, false, true, 16 | 64>), groups, G, S, lds, s, mp, a, G, invS);
        F2A_LAUNCH_GROUPS((k_p1<3, 1, 2, 2, false, true, 64>), groups, G, S, lds, s, mp, a, G, invS);
    default:
        if (in) F2A_LAUNCH_GROUPS((k_p1<1, 1, 2, 2, false, true, 16 | 64>), groups, G, S, lds, s, mp, a, G, invS);
        F2A_LAUNCH_GROUPS((k_p1<1, 1, 2, 2, false, true, 64>), groups, G, S, lds, s, mp, a, G, invS);
    }
}

hipError_t launch_p2h(const MeshPlanDev &mp, const P2Args &a, hipStream_t s)
{
    const int L = a.nl - 1;
    // single-use streams non-temporal (FESOM2_NT bit 1), 16-byte loads of the stride-nl area
    const bool NT = (knob("FESOM2_NT", 6) & 2) != 0;
    const bool pair = knob("FESOM2_NL_PAIR", 1) != 0;
    if (odd_pairs(L)) {
        const int S = (L + 1) / 2, G = plan_columns(S, mp);
        const long groups = (long)(a.count + G - 1) / G * a.tr.n;
        const size_t lds = (size_t)G * sizeof(NodeRec);
        const float invS = 1.0f / (float)S;
#if F2A_TUNING
        if (!NT) F2A_LAUNCH_GROUPS((k_p2h<2, 4, false, true, true>), groups, G, S, lds, s, mp, a, G, invS);
        if (knob("FESOM2_P2H_BATCH", 4) == 6) F2A_LAUNCH_GROUPS((k_p2h<2, 6, true, true, true>), groups, G, S, lds, s, mp, a, G, invS);
        if (knob("FESOM2_P2H_BATCH", 4) == 8) F2A_LAUNCH_GROUPS((k_p2h<2, 8, true, true, true>), groups, G, S, lds, s, mp, a, G, invS);
#endif
        F2A_LAUNCH_GROUPS((k_p2h<2, 4, true, true, true>), groups, G, S, lds, s, mp, a, G, invS);
    }
    const int C = levels_per_thread(L), S = L / C, G = plan_columns(S, mp);
    const long groups = (long)(a.count + G - 1) / G * a.tr.n;
    const float invS = 1.0f / (float)S;
    const size_t lds = (size_t)G * sizeof(NodeRec);
#if F2A_TUNING
    if (C == 2) {
        // FESOM2_P2H_BATCH: edge gathers per round trip (6 or 8: a structured node's 6 edges in one)
        if (NT && pair && knob("FESOM2_P2H_BATCH", 4) == 6)
            F2A_LAUNCH_GROUPS((k_p2h<2, 6, true, true>), groups, G, S, lds, s, mp, a, G, invS);
        if (NT && pair && knob("FESOM2_P2H_BATCH", 4) == 8)
            F2A_LAUNCH_GROUPS((k_p2h<2, 8, true, true>), groups, G, S, lds, s, mp, a, G, invS);
        if (NT && !pair) F2A_LAUNCH_GROUPS((k_p2h<2, 4, true>), groups, G, S, lds, s, mp, a, G, invS);
        if (!NT && pair) F2A_LAUNCH_GROUPS((k_p2h<2, 4, false, true>), groups, G, S, lds, s, mp, a, G, invS);
        if (!NT) F2A_LAUNCH_GROUPS((k_p2h<2, 4, false>), groups, G, S, lds, s, mp, a, G, invS);
    }
    if (!NT) F2A_LAUNCH_GROUPS((k_p2h<1, 4, false>), groups, G, S, lds, s, mp, a, G, invS);
#else
    (void)NT, (void)pair;
#endif
    if (C == 2) F2A_LAUNCH_GROUPS((k_p2h<2, 4, true, true>), groups, G, S, lds, s, mp, a, G, invS);
    F2A_LAUNCH_GROUPS((k_p2h<1, 4, true>), groups, G, S, lds, s, mp, a, G, invS);
}

hipError_t launch_p2_fused(const MeshPlanDev &mp, const P2Args &a, hipStream_t s)
{
    const int L = a.nl - 1;
    // levels per thread of the node kernel: FESOM2_P2_CPT (tuning build; default as the other kernels)
    const int C = (L % 2 == 0 && knob("FESOM2_P2_CPT", levels_per_thread(L)) == 2) ? 2 : 1;
    const int S = L / C, G = plan_columns(S, mp);
    const long groups = (long)(a.count + G - 1) / G * a.tr.n;
    const float invS = 1.0f / (float)S;
    const size_t lds = (size_t)G * sizeof(NodeRec);
#if F2A_TUNING
    const int KB = knob("FESOM2_P2_BATCH", 4);
    const bool NT = (knob("FESOM2_NT", 6) & 2) != 0;
    if (C == 2 && NT && KB == 2) F2A_LAUNCH_GROUPS((k_p2<2, 2, true>), groups, G, S, lds, s, mp, a, G, invS);
    if (!NT || KB != 4) {
        if (C == 2 && KB == 8) F2A_LAUNCH_GROUPS((k_p2<2, 8, false>), groups, G, S, lds, s, mp, a, G, invS);
        if (C == 2) F2A_LAUNCH_GROUPS((k_p2<2, 4, false>), groups, G, S, lds, s, mp, a, G, invS);
        if (KB == 8) F2A_LAUNCH_GROUPS((k_p2<1, 8, false>), groups, G, S, lds, s, mp, a, G, invS);
        if (KB == 2) F2A_LAUNCH_GROUPS((k_p2<1, 2, false>), groups, G, S, lds, s, mp, a, G, invS);
        F2A_LAUNCH_GROUPS((k_p2<1, 4, false>), groups, G, S, lds, s, mp, a, G, invS);
    }
#endif
    // edge gathers in batches of 4, single-use streams non-temporal (measured -2 %)
    if (C == 2) F2A_LAUNCH_GROUPS((k_p2<2, 4, true>), groups, G, S, lds, s, mp, a, G, invS);
    F2A_LAUNCH_GROUPS((k_p2<1, 4, true>), groups, G, S, lds, s, mp, a, G, invS);
}

hipError_t launch_b3v_cols(int n_owned, int nl, const int *nlev, const real *plus, const real *minus, real *adf_v,
                           hipStream_t s)
{
    const int L = nl - 1;
    const bool odd = L % 2 == 1;
    if (odd && L < 3) return launch_b3v(n_owned, nl, nlev, plus, minus, adf_v, s);
    const int S = (L + 1) / 2, G = group_columns(S);
    const long groups = (n_owned + G - 1) / G;
    const float invS = 1.0f / (float)S;
    if (odd) F2A_LAUNCH_GROUPS((k_b3v_g<2, true>), groups, G, S, 0, s, n_owned, L, G, invS, nlev, plus, minus, adf_v);
    F2A_LAUNCH_GROUPS((k_b3v_g<2, false>), groups, G, S, 0, s, n_owned, L, G, invS, nlev, plus, minus, adf_v);
}

hipError_t launch_c_fused(const MeshPlanDev &mp, const P2Args &a, hipStream_t s)
{
    const int L = a.nl - 1;
    const bool odd = L % 2 == 1;
    if (odd && L < 3) return hipErrorInvalidValue;
    const int S = (L + 1) / 2, G = plan_columns(S, mp);
    const long groups = (a.count + G - 1) / G;
    const float invS = 1.0f / (float)S;
    const size_t lds = (size_t)G * sizeof(NodeRec);
#if F2A_TUNING
    // FESOM2_C_BATCH = 2: edge gathers in batches of 2 (fewer VGPRs, more resident waves)
    if (knob("FESOM2_C_BATCH", 4) == 2) {
        if (odd) F2A_LAUNCH_GROUPS((k_c<2, 2, true>), groups, G, S, lds, s, mp, a, G, invS);
        F2A_LAUNCH_GROUPS((k_c<2, 2, false>), groups, G, S, lds, s, mp, a, G, invS);
    }
#endif
    if (odd) F2A_LAUNCH_GROUPS((k_c<2, 4, true>), groups, G, S, lds, s, mp, a, G, invS);
    F2A_LAUNCH_GROUPS((k_c<2, 4, false>), groups, G, S, lds, s, mp, a, G, invS);
}

// packed b3h over descriptors [d0, d1) of a list (k_b3h_p), or false if packing is off for this L.
// Production form: two level-pair slots per thread, fct_adf_h non-temporal, and on a regular list
// (reg.x > 0: every edge the same slot count) no descriptor loads.
static bool launch_b3h_packed(const int2 *desc, const unsigned short *off, const int4 *einfo, int cap, int d0, int d1,
                              int nl, const real *plus, const real *minus, real *adf_h, const Tracers &tr,
                              hipStream_t s, hipError_t *err, int4 reg = make_int4(0, 0, 0, 0))
{
    const int L = nl - 1;
    if (!desc || !knob("FESOM2_B3H_PACK", 1) || !(L % 2 == 0 || odd_pairs(L))) return false;
    const long groups = (long)(d1 - d0) * tr.n;
    init_swizzle();
    *err = hipSuccess;
    if (groups <= 0) return true;
    const int4 none = make_int4(0, 0, 0, 0);
#if F2A_TUNING
    // slots per thread (FESOM2_B3HP_H 1 or 4: even L, non-temporal only, the block must cover the
    // capacity), cached fct_adf_h (FESOM2_B3H_NT=0), descriptor loads on regular lists (FESOM2_B3HP_REG=0)
    const bool NT = knob("FESOM2_B3H_NT", 1) != 0;
    int H = knob("FESOM2_B3HP_H", 2);
    if ((H != 1 && H != 4) || (L % 2) || !NT || (H == 1 && cap > 1024)) H = 2;
    if (H != 2 || !NT || !knob("FESOM2_B3HP_REG", 1)) {
        const dim3 grid((unsigned)groups), block((cap + H - 1) / H);
        if (H == 1)
            hipLaunchKernelGGL((k_b3h_p<true, false, 1>), grid, block, 0, s, desc + d0, off, einfo, L, plus, minus, adf_h, tr, none);
        else if (H == 4)
            hipLaunchKernelGGL((k_b3h_p<true, false, 4>), grid, block, 0, s, desc + d0, off, einfo, L, plus, minus, adf_h, tr, none);
        else if (L % 2)
            hipLaunchKernelGGL((k_b3h_p<true, true>), grid, block, 0, s, desc + d0, off, einfo, L, plus, minus, adf_h, tr, none);
        else if (NT)
            hipLaunchKernelGGL((k_b3h_p<true, false>), grid, block, 0, s, desc + d0, off, einfo, L, plus, minus, adf_h, tr, none);
        else
            hipLaunchKernelGGL((k_b3h_p<false, false>), grid, block, 0, s, desc + d0, off, einfo, L, plus, minus, adf_h, tr, none);
        *err = hipGetLastError();
        return true;
    }
#endif
    const dim3 grid((unsigned)groups), block((cap + 1) / 2);
    // a pass whose fct_adf_h fits the Infinity Cache (Tracers::order bit 3): the limited fluxes as
    // plain stores, which c-horizontal then reads from the cache (tuning: FESOM2_B3H_STPLAIN forces it)
    const bool plain = (tr.order & 8) != 0 || knob("FESOM2_B3H_STPLAIN", 0) != 0;
#define F2A_B3HP(ODD, REG, PLAIN, R)                                                                                   \
    hipLaunchKernelGGL((k_b3h_p<true, ODD, 2, REG, !(PLAIN)>), grid, block, 0, s, desc + d0, off, einfo, L, plus, minus, \
                       adf_h, tr, R)
    if (reg.x > 0) {
        if (L % 2) {
            if (plain) F2A_B3HP(true, true, true, reg);
            else F2A_B3HP(true, true, false, reg);
        } else {
            if (plain) F2A_B3HP(false, true, true, reg);
            else F2A_B3HP(false, true, false, reg);
        }
    } else if (L % 2) {
        if (plain) F2A_B3HP(true, false, true, none);
        else F2A_B3HP(true, false, false, none);
    } else {
        if (plain) F2A_B3HP(false, false, true, none);
        else F2A_B3HP(false, false, false, none);
    }
#undef F2A_B3HP
    *err = hipGetLastError();
    return true;
}

hipError_t launch_b3h_fused(const MeshPlanDev &mp, int nl, int begin, int count, const real *plus,
                            const real *minus, real *adf_h, const Tracers &tr, hipStream_t s)
{
    // packed by depth: the plan's descriptors for exactly these edge ranges
    int d0 = -1, d1 = -1, sl = 0;  // sl: regular slot count of the edge range, if any
    const int ni = mp.n_edge_interior;
    if (begin == 0 && count == mp.n_edges) d0 = 0, d1 = mp.b3p_ndesc, sl = ni == mp.n_edges ? mp.b3p_slots_int : 0;
    else if (begin == 0 && count == ni) d0 = 0, d1 = mp.b3p_nint, sl = mp.b3p_slots_int;
    else if (begin == ni && begin + count == mp.n_edges) d0 = mp.b3p_nint, d1 = mp.b3p_ndesc, sl = mp.b3p_slots_bnd;
    const int4 reg = sl > 0 ? make_int4(std::min(kB3hPackEdges, mp.b3p_cap / sl), sl, begin, count) : make_int4(0, 0, 0, 0);
    hipError_t err;
    if (d0 >= 0 && launch_b3h_packed(mp.b3p_desc, mp.b3p_off, mp.p_edge_info, mp.b3p_cap, d0, d1, nl, plus, minus,
                                     adf_h, tr, s, &err, reg))
        return err;
    return launch_b3h_edges(mp.p_edge_info + begin, count, nl, plus, minus, adf_h, tr, s);
}

hipError_t launch_b3h_ext(const MeshPlanDev &mp, int nl, const real *plus, const real *minus, real *adf_h,
                          const Tracers &tr, hipStream_t s)
{
    if (mp.n_ext_interior == 0) return hipSuccess;
    if (!mp.p_edge_ext) return hipErrorInvalidValue;
    hipError_t err;
    const int4 reg = mp.b3x_slots > 0 ? make_int4(std::min(kB3hPackEdges, mp.b3x_cap / mp.b3x_slots), mp.b3x_slots, 0,
                                                  mp.n_ext_interior)
                                      : make_int4(0, 0, 0, 0);
    if (launch_b3h_packed(mp.b3x_desc, mp.b3x_off, mp.p_edge_ext, mp.b3x_cap, 0, mp.b3x_ndesc, nl, plus, minus, adf_h,
                          tr, s, &err, reg))
        return err;
    return launch_b3h_edges(mp.p_edge_ext, mp.n_ext_interior, nl, plus, minus, adf_h, tr, s);
}

// b3-horizontal over an explicit edge list: two edge groups per block (every einfo load, then every
// data load of both groups issued before use), fct_adf_h non-temporal
hipError_t launch_b3h_edges(const int4 *ei, int count, int nl, const real *plus, const real *minus,
                            real *adf_h, const Tracers &tr, hipStream_t s)
{
    const int L = nl - 1;
    if (odd_pairs(L)) {
        const int S = (L + 1) / 2, G = group_columns(S);
        const long ug = ((count + G - 1) / G + 1) / 2 * tr.n;
        F2A_LAUNCH_GROUPS((k_b3h_u<2, 2, true, true>), ug, G, S, 0, s, ei, count, L, G, 1.0f / (float)S, plus, minus,
                          adf_h, tr);
    }
    int C = levels_per_thread(L);
    const int S0 = L / C, G0 = group_columns(S0);
    const long groups0 = (count + G0 - 1) / G0;
#if F2A_TUNING
    // 4 levels per thread (FESOM2_B3H_CPT=4), U edge groups per block (FESOM2_B3H_U), cached
    // fct_adf_h (FESOM2_B3H_NT=0)
    if (C == 2 && L % 4 == 0 && knob("FESOM2_B3H_CPT", 2) == 4) C = 4;
    const int U = knob("FESOM2_B3H_U", 2);
    const bool NT = knob("FESOM2_B3H_NT", 1) != 0;
    if (C == 4 || U != 2 || !NT) {
        const int S = L / C, G = group_columns(S);
        const long groups = (count + G - 1) / G;
        const float invS = 1.0f / (float)S;
        const long tg = groups * tr.n, ug = (groups + U - 1) / U * tr.n;
        if (C == 4) F2A_LAUNCH_GROUPS(k_b3h_g<4>, tg, G, S, 0, s, ei, count, L, G, invS, plus, minus, adf_h, tr);
        if (C == 2 && NT && U == 4) F2A_LAUNCH_GROUPS((k_b3h_u<2, 4, true>), ug, G, S, 0, s, ei, count, L, G, invS, plus, minus, adf_h, tr);
        if (C == 2 && NT && U == 8) F2A_LAUNCH_GROUPS((k_b3h_u<2, 8, true>), ug, G, S, 0, s, ei, count, L, G, invS, plus, minus, adf_h, tr);
        if (C == 2 && NT && U == 1) F2A_LAUNCH_GROUPS((k_b3h_u<2, 1, true>), tg, G, S, 0, s, ei, count, L, G, invS, plus, minus, adf_h, tr);
        if (C == 2 && !NT && U == 2) F2A_LAUNCH_GROUPS((k_b3h_u<2, 2, false>), ug, G, S, 0, s, ei, count, L, G, invS, plus, minus, adf_h, tr);
        if (C == 2) F2A_LAUNCH_GROUPS(k_b3h_g<2>, tg, G, S, 0, s, ei, count, L, G, invS, plus, minus, adf_h, tr);
        if (U == 4 && NT) F2A_LAUNCH_GROUPS((k_b3h_u<1, 4, true>), ug, G, S, 0, s, ei, count, L, G, invS, plus, minus, adf_h, tr);
        F2A_LAUNCH_GROUPS(k_b3h_g<1>, tg, G, S, 0, s, ei, count, L, G, invS, plus, minus, adf_h, tr);
    }
#endif
    const float invS = 1.0f / (float)S0;
    const long ug = (groups0 + 1) / 2 * tr.n;
    if (C == 2) F2A_LAUNCH_GROUPS((k_b3h_u<2, 2, true>), ug, G0, S0, 0, s, ei, count, L, G0, invS, plus, minus, adf_h, tr);
    F2A_LAUNCH_GROUPS((k_b3h_u<1, 2, true>), ug, G0, S0, 0, s, ei, count, L, G0, invS, plus, minus, adf_h, tr);
}

hipError_t launch_p2_iter(const MeshPlanDev &mp, const P2IterArgs &a, hipStream_t s)
{
    const int L = a.nl - 1, C = levels_per_thread(L), S = L / C, G = plan_columns(S, mp);
    const long groups = (long)(a.count + G - 1) / G * a.tr.n;
    const float invS = 1.0f / (float)S;
    const size_t lds = (size_t)G * sizeof(NodeRec);
    if (C == 2) F2A_LAUNCH_GROUPS((k_p2_iter<2>), groups, G, S, lds, s, mp, a, G, invS);
    F2A_LAUNCH_GROUPS((k_p2_iter<1>), groups, G, S, lds, s, mp, a, G, invS);
}

hipError_t launch_b3h_iter(const MeshPlanDev &mp, int nl, const real *plus, const real *minus, real *adf_h,
                           real *adf_h2, const Tracers &tr, hipStream_t s)
{
    const int L = nl - 1, C = levels_per_thread(L), S = L / C, G = plan_columns(S, mp);
    const long groups = (long)(mp.n_edges + G - 1) / G * tr.n;
    const float invS = 1.0f / (float)S;
    if (C == 2)
        F2A_LAUNCH_GROUPS((k_b3h_iter<2>), groups, G, S, 0, s, mp.p_edge_info, mp.n_edges, L, G, invS, plus, minus,
                          adf_h, adf_h2, tr);
    F2A_LAUNCH_GROUPS((k_b3h_iter<1>), groups, G, S, 0, s, mp.p_edge_info, mp.n_edges, L, G, invS, plus, minus, adf_h,
                      adf_h2, tr);
}

hipError_t launch_halo_pack(const int *nodes, int count, int L, int ntr, size_t stride, const real *plus,
                            const real *minus, real *buf, hipStream_t s)
{
    F2A_LAUNCH(k_pack, (long)count * ntr, 0, s, nodes, count, L, ntr, stride, plus, minus, buf);
}

hipError_t launch_halo_unpack(const int *nodes, int count, int L, int ntr, size_t stride, const real *buf,
                              real *plus, real *minus, hipStream_t s)
{
    F2A_LAUNCH(k_unpack, (long)count * ntr, 0, s, nodes, count, L, ntr, stride, buf, plus, minus);
}

}  // namespace f2a
