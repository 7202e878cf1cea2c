// fct_ale_variants.hip -- measured alternatives to the production fused kernels (all exact, all
// opt-in through environment switches; DESIGN.md §3 records why each is not the default):
//   * k_p1e  FESOM2_P1_EDGE=1   phase 1 gathering the cluster along the edge list
//   * k_p1s  FESOM2_P1_STAGE=1  phase 1 with the block's cluster columns staged in LDS
//   * k_p2f  FESOM2_FUSE_B3H=1  b3-horizontal folded into the node kernel (arrival counters)
//   * k_p2_b3h_chunk  FESOM2_P2_CHUNK + FESOM2_P2_MERGE  chunked phase 2, merged boundaries
//   * k_p2w  FESOM2_P2_WF=1     phase 2 as one persistent launch with per-tile hand-offs
//   * k_p2hf FESOM2_P2H_FUSE=1  b3-horizontal folded into c-horizontal on the split pass
//   * k_b3h_n FESOM2_B3H_NODE=1 b3-horizontal node-centric over the owner order
// Compiled into the tuning build only (make tuning, F2A_TUNING=1); the product library has none.
#include "f2a_device.hpp"

#if !F2A_TUNING
#error "fct_ale_variants.hip belongs to the tuning build (make tuning)"
#endif

namespace f2a {

// Phase 2, horizontal half with b3-horizontal folded in (FESOM2_P2H_FUSE): c-horizontal over the
// node's edges with each raw fct_adf_h limited in-thread from both endpoints' plus/minus, so the
// separate b3h pass (read + write of fct_adf_h, plus/minus gathers) and p2h's re-read of the limited
// flux become one read of the raw flux per endpoint.  The limited flux is stored in place once, by
// the endpoint that reads the raw flux last: after the block barrier (all raw reads of the block
// done) one thread per (column, edge) bumps the edge's arrival counter -- counters only ever grow by
// the edge's owned endpoints, two per pass, so an odd old value marks the second arriver and no
// reset is needed -- and a halo endpoint never arrives, so the owned one writes.  The writer loads
// the raw flux and the other endpoint's plus/minus again (L2-resident: its block just read them).
template <int C, int KB, bool NT, bool ODD>
__global__ __launch_bounds__(1024) void k_p2hf(MeshPlanDev mp, P2Args a, int G, float invS)
{
    extern __shared__ real lds[];  // NodeRec[G] | writer masks[G]
    const int L = a.nl - 1, S = (L + C - 1) / C;
    int tr;
    const int first = group_tracer(a.tr.n, tr, c_tracer_major & 4) * G;
    if (tr) {
        a.plus += tr * a.tr.node;
        a.minus += tr * a.tr.node;
        a.del_h += tr * a.tr.node;
        a.adf_h += tr * a.tr.edge;
        a.edge_cnt += (size_t)tr * mp.n_edges;
    }
    unsigned *wmask = reinterpret_cast<unsigned *>(reinterpret_cast<NodeRec *>(lds) + G);
    if ((int)threadIdx.x < G) wmask[threadIdx.x] = 0u;
    const int ncol = min(G, a.count - first);
    const NodeRec *recs = stage_records(a.nodes, first, ncol, lds);  // (its barrier also orders wmask)
    int j, u;
    slot_of(threadIdx.x, S, invS, j, u);
    const int z0 = C * u;
    const bool last1 = ODD && z0 + 1 == L;
    const bool col = j < ncol;
    NodeInfo ni{};
    if (col) ni = recs[j].info;
    const int nw = col ? max(0, min(C, ni.Ln - z0)) : 0;
    const int ne = col ? ni.e1 - ni.e0 : 0;
    real pn[C], mn[C], dh[C];
    size_t b = 0;
    if (nw > 0) {
        b = (size_t)ni.n * L + z0;
        const size_t ab = (size_t)ni.n * a.nl + z0;
        ldo<C, ODD>(a.plus + b, pn, last1);
        ldo<C, ODD>(a.minus + b, mn, last1);
        ldo_s<C, NT, ODD>(a.del_h + b, dh, last1);
        real dta[C];
        if constexpr (C == 2) {  // area: one 16-B load at 8-B alignment (ld_nl)
            const f2a_d2u t = NT ? __builtin_nontemporal_load(reinterpret_cast<const f2a_d2u *>(a.area + ab))
                                 : *reinterpret_cast<const f2a_d2u *>(a.area + ab);
            dta[0] = a.dt / t.x;
            dta[1] = nw >= 2 ? a.dt / t.y : 0.;
        } else {
#pragma unroll
            for (int c = 0; c < C; c++) dta[c] = c < nw ? a.dt / ld1_s<NT>(a.area + ab + c) : 0.;
        }
        auto add = [&](int c, real h, int second, int) {
            dh[c] = second ? dh[c] - h * dta[c] : dh[c] + h * dta[c];  // docs/refactoring.md:311-312
        };
        for_edges_limited<C, KB, ODD>(recs[j].edge, 0, min(ne, kRecEdge), a.adf_h, a.plus, a.minus, pn, mn, z0, L,
                                      add, last1);
        if (ne > kRecEdge)
            for_edges_limited<C, KB, ODD>(mp.p_edges, ni.e0 + kRecEdge, ni.e1, a.adf_h, a.plus, a.minus, pn, mn, z0, L,
                                          add, last1);
    }
    __syncthreads();  // every raw fct_adf_h read of the block is done
    const int abl = c_ablate;  // timing-only experiments: 16 static writer (racy), 32 no writer
    for (int k = u; k < ne; k += S) {
        const EdgeRef er = k < kRecEdge ? recs[j].edge[k] : mp.p_edges[ni.e0 + k];
        if ((abl & 16) ? !(er.code & 1)
                       : (er.other >= a.n_owned || (atomicAdd(reinterpret_cast<unsigned *>(a.edge_cnt) + er.edge, 1u) & 1u)))
            atomicOr(&wmask[j], 1u << k);
    }
    __syncthreads();
    if (nw <= 0) return;
    stv_s<C, NT>(a.del_h + b, dh, nw);
    unsigned mine = (abl & 32) ? 0u : wmask[j];
    while (mine) {  // the edges this column writes, KB at a time
        int ks[KB];
#pragma unroll
        for (int q = 0; q < KB; q++) {
            ks[q] = mine ? __builtin_ctz(mine) : -1;
            if (mine) mine &= mine - 1;
        }
        EdgeRef er[KB];
        real h[KB][C], po[KB][C], mo[KB][C];
#pragma unroll
        for (int q = 0; q < KB; q++) {
            er[q] = ks[q] < 0 ? EdgeRef{0, 0, 0} : (ks[q] < kRecEdge ? recs[j].edge[ks[q]] : mp.p_edges[ni.e0 + ks[q]]);
            if (z0 < (er[q].code >> 1)) {
                ldo_s<C, NT, ODD>(a.adf_h + (size_t)er[q].edge * L + z0, h[q], last1);
                ldo<C, ODD>(a.plus + (size_t)er[q].other * L + z0, po[q], last1);
                ldo<C, ODD>(a.minus + (size_t)er[q].other * L + z0, mo[q], last1);
            }
        }
#pragma unroll
        for (int q = 0; q < KB; q++) {
            const int lev = er[q].code >> 1, second = er[q].code & 1;
            if (z0 >= lev) continue;
            real out[C];
#pragma unroll
            for (int c = 0; c < C; c++)
                out[c] = (second ? b3h_factor(h[q][c], po[q][c], mo[q][c], pn[c], mn[c])
                                 : b3h_factor(h[q][c], pn[c], mn[c], po[q][c], mo[q][c])) * h[q][c];
            stv_s<C, NT>(a.adf_h + (size_t)er[q].edge * L + z0, out, min(C, lev - z0));
        }
    }
}

// b3-horizontal, node-centric: column j of the block is processing position k and limits the edges
// k owns (first visited endpoint, MeshPlanDev::p_edge_owner[p_owner_cum[k] ..)), all incident to
// its node n: n's plus/minus are loaded once, per edge only fct_adf_h (non-temporal) and the other
// endpoint's plus/minus -- 3 loads per edge instead of 5.  Every edge is written once, by its
// owner, and read by nobody else in the launch.  Same b3h_factor arithmetic as k_b3h_u.
template <int C, int EB, bool NT, bool ODD>
__global__ __launch_bounds__(1024) void k_b3h_n(const NodeInfo *__restrict__ info, const int *__restrict__ owner_cum,
                                                const int4 *__restrict__ eown, int n_pos, int L, int G, float invS,
                                                const real *__restrict__ plus, const real *__restrict__ minus,
                                                real *__restrict__ adf_h, Tracers trs)
{
    int tr;
    const int first = group_tracer(trs.n, tr, c_tracer_major & 2) * G;
    plus += tr * trs.node;
    minus += tr * trs.node;
    adf_h += tr * trs.edge;
    int j, u;
    slot_of(threadIdx.x, (L + C - 1) / C, invS, j, u);
    const int k = first + j;
    if (j >= G || k >= n_pos) return;
    const int z0 = C * u;
    const bool last1 = ODD && z0 + 1 == L;
    const int e0 = owner_cum[k], e1 = owner_cum[k + 1];
    if (e0 >= e1) return;
    const int n = info[k].n;
    real po[C], mo[C];
    ldo<C, ODD>(plus + (size_t)n * L + z0, po, last1);
    ldo<C, ODD>(minus + (size_t)n * L + z0, mo, last1);
    for (int q0 = e0; q0 < e1; q0 += EB) {
        int4 ei[EB];
#pragma unroll
        for (int q = 0; q < EB; q++) ei[q] = q0 + q < e1 ? eown[q0 + q] : make_int4(0, 0, 0, 0);
        real f[EB][C], px[EB][C], mx[EB][C];
#pragma unroll
        for (int q = 0; q < EB; q++) {
            if (z0 < ei[q].z) {
                const int o = ei[q].x == n ? ei[q].y : ei[q].x;
                ldo_s<C, NT, ODD>(adf_h + (size_t)ei[q].w * L + z0, f[q], last1);
                ldo<C, ODD>(plus + (size_t)o * L + z0, px[q], last1);
                ldo<C, ODD>(minus + (size_t)o * L + z0, mx[q], last1);
            }
        }
#pragma unroll
        for (int q = 0; q < EB; q++) {
            const int nw = min(C, ei[q].z - z0);
            if (nw <= 0) continue;
            const bool own_first = ei[q].x == n;  // node1 of the edge (docs/refactoring.md:246-257)
            real out[C];
#pragma unroll
            for (int c = 0; c < C; c++)
                out[c] = (own_first ? b3h_factor(f[q][c], po[c], mo[c], px[q][c], mx[q][c])
                                    : b3h_factor(f[q][c], px[q][c], mx[q][c], po[c], mo[c])) * f[q][c];
            stv_s<C, NT>(adf_h + (size_t)ei[q].w * L + z0, out, nw);
        }
    }
}

hipError_t launch_p2hf(const MeshPlanDev &mp, const P2Args &a, hipStream_t s)
{
    const int L = a.nl - 1;
    const bool odd = odd_pairs(L);
    const int C = odd ? 2 : levels_per_thread(L), S = (L + C - 1) / C, G = group_columns(S);
    const long groups = (long)(a.count + G - 1) / G * a.tr.n;
    const float invS = 1.0f / (float)S;
    const size_t lds = (size_t)G * sizeof(NodeRec) + G * sizeof(unsigned);
    const bool NT = (knob("FESOM2_NT", 6) & 2) != 0;
    const int KB = knob("FESOM2_P2HF_KB", 2);
    if (odd) {
        if (NT) F2A_LAUNCH_GROUPS((k_p2hf<2, 2, true, true>), groups, G, S, lds, s, mp, a, G, invS);
        F2A_LAUNCH_GROUPS((k_p2hf<2, 2, false, true>), groups, G, S, lds, s, mp, a, G, invS);
    }
    if (C == 2) {
        if (KB == 4) F2A_LAUNCH_GROUPS((k_p2hf<2, 4, true, false>), groups, G, S, lds, s, mp, a, G, invS);
        if (KB == 1) F2A_LAUNCH_GROUPS((k_p2hf<2, 1, true, false>), groups, G, S, lds, s, mp, a, G, invS);
        if (NT) F2A_LAUNCH_GROUPS((k_p2hf<2, 2, true, false>), groups, G, S, lds, s, mp, a, G, invS);
        F2A_LAUNCH_GROUPS((k_p2hf<2, 2, false, false>), groups, G, S, lds, s, mp, a, G, invS);
    }
    F2A_LAUNCH_GROUPS((k_p2hf<1, 2, false, false>), groups, G, S, lds, s, mp, a, G, invS);
}
hipError_t launch_b3h_nodes(const MeshPlanDev &mp, int nl, int owned_edges, int n_edges, const real *plus,
                            const real *minus, real *adf_h, const Tracers &tr, hipStream_t s)
{
    const int L = nl - 1, N = mp.n_owned;
    if (!mp.p_owner_cum || !mp.node_info) return hipErrorInvalidValue;
    const bool odd = L % 2 == 1;
    const int C = (L % 2 == 0 || odd_pairs(L)) ? 2 : 1;
    const int S = (L + C - 1) / C, G = group_columns(S);
    const long groups = (long)(N + G - 1) / G * tr.n;
    const float invS = 1.0f / (float)S;
    const int EB = knob("FESOM2_B3HN_EB", 2);
    auto go = [&]() -> hipError_t {
        if (C == 2 && !odd) {
            if (EB == 1) F2A_LAUNCH_GROUPS((k_b3h_n<2, 1, true, false>), groups, G, S, 0, s, mp.node_info, mp.p_owner_cum,
                                           mp.p_edge_owner, N, L, G, invS, plus, minus, adf_h, tr);
            if (EB == 3) F2A_LAUNCH_GROUPS((k_b3h_n<2, 3, true, false>), groups, G, S, 0, s, mp.node_info, mp.p_owner_cum,
                                           mp.p_edge_owner, N, L, G, invS, plus, minus, adf_h, tr);
            F2A_LAUNCH_GROUPS((k_b3h_n<2, 2, true, false>), groups, G, S, 0, s, mp.node_info, mp.p_owner_cum,
                              mp.p_edge_owner, N, L, G, invS, plus, minus, adf_h, tr);
        }
        if (C == 2)
            F2A_LAUNCH_GROUPS((k_b3h_n<2, 2, true, true>), groups, G, S, 0, s, mp.node_info, mp.p_owner_cum,
                              mp.p_edge_owner, N, L, G, invS, plus, minus, adf_h, tr);
        F2A_LAUNCH_GROUPS((k_b3h_n<1, 2, true, false>), groups, G, S, 0, s, mp.node_info, mp.p_owner_cum,
                          mp.p_edge_owner, N, L, G, invS, plus, minus, adf_h, tr);
    };
    const hipError_t e = go();
    if (e != hipSuccess || owned_edges >= n_edges) return e;
    // edges without an owned endpoint (none in a FESOM partition): edge-centric
    return launch_b3h_edges(mp.p_edge_owner + owned_edges, n_edges - owned_edges, nl, plus, minus, adf_h, tr, s);
}


// Phase-1 edge loop that also gathers the cluster (MeshPlanDev::edge_cluster): per edge the raw
// flux and the other endpoint's LO/ttf, kBatch edges at a time; b1-horizontal sums in ascending
// edge order (f), max/min(LO, ttf) of the neighbour on the edge's levels into vx/vn.
template <int C, int kBatch, class F>
__device__ __forceinline__ void for_edges_cluster(const EdgeRef *__restrict__ edges, int e0, int e1,
                                                  const real *__restrict__ adf_h,
                                                  const real *__restrict__ LO,
                                                  const real *__restrict__ ttf, int z0, int L,
                                                  real (&vx)[C], real (&vn)[C], F &&f)
{
    for (int k0 = e0; k0 < e1; k0 += kBatch) {
        EdgeRef er[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; k++) er[k] = (k0 + k < e1) ? edges[k0 + k] : EdgeRef{0, 0, 0};
        real h[kBatch][C], lo[kBatch][C], tt[kBatch][C];
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            if (z0 < (er[k].code >> 1)) {
                ldv<C>(adf_h + (size_t)er[k].edge * L + z0, h[k]);
                ldv<C>(LO + (size_t)er[k].other * L + z0, lo[k]);
                ldv<C>(ttf + (size_t)er[k].other * L + z0, tt[k]);
            }
        }
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            const int lev = er[k].code >> 1;
#pragma unroll
            for (int c = 0; c < C; c++)
                if (z0 + c < lev) {
                    f(c, h[k][c], er[k].code & 1);
                    vx[c] = RMAX(vx[c], RMAX(lo[k][c], tt[k][c]));
                    vn[c] = RMIN(vn[c], RMIN(lo[k][c], tt[k][c]));
                }
        }
    }
}

// Phase 1 with the cluster taken along the edge list (see for_edges_cluster): one gather loop of
// three columns per edge instead of a cluster loop and an edge loop, and the node's own LO/ttf
// loaded once for both its cluster term and b2.
template <int VLIMIT, int C, int EB>
__global__ __launch_bounds__(1024) void k_p1e(MeshPlanDev mp, P1Args a, int G, float invS)
{
    extern __shared__ real lds[];  // tvert max | tvert min | NodeRec[G]
    const int L = a.nl - 1, S = L / C;
    const int t = threadIdx.x;
    int tr;
    const int first = group_tracer(a.tr.n, tr, c_tracer_major & 1) * G;
    if (tr) {
        a.ttf += tr * a.tr.node;
        a.LO += tr * a.tr.node;
        a.plus += tr * a.tr.node;
        a.minus += tr * a.tr.node;
        a.adf_v += tr * a.tr.lev;
        a.adf_h += tr * a.tr.edge;
    }
    const int ncol = min(G, a.n_owned - first);
    const NodeRec *recs = stage_records(mp.node_rec, first, ncol, lds + 2 * G * L);
    int j, u;
    slot_of(t, S, invS, j, u);
    const int z0 = C * u;
    const bool col = j < ncol;
    NodeInfo ni{};
    if (col) ni = recs[j].info;
    const int Ln = ni.Ln;
    const int nw = col ? max(0, min(C, Ln - z0)) : 0;
    real vx[C], vn[C], p[C], m[C], lo[C], tt[C];
#pragma unroll
    for (int c = 0; c < C; c++) vx[c] = vn[c] = p[c] = m[c] = lo[c] = tt[c] = 0.;
    size_t b = 0, ab = 0;
    if (nw > 0) {
        b = (size_t)ni.n * L + z0;
        ab = (size_t)ni.n * a.nl + z0;
        ldv<C>(a.LO + b, lo);
        ldv<C>(a.ttf + b, tt);
        real v[C + 1];
#pragma unroll
        for (int c = 0; c <= C; c++) v[c] = (c == 0 || c < nw + 1) ? a.adf_v[ab + c] : 0.;
#pragma unroll
        for (int c = 0; c < C; c++) {
            p[c] = RMAX(0., v[c]) + RMAX(0., -v[c + 1]);  // b1-vertical, reference.cpp:393-399
            m[c] = RMIN(0., v[c]) + RMIN(0., -v[c + 1]);
            const bool dry = z0 + c >= ni.zdry;
            vx[c] = dry ? -a.big : -INFINITY;
            vn[c] = dry ? a.big : INFINITY;
            if (z0 + c < ni.self_lev) {  // the node itself
                vx[c] = RMAX(vx[c], RMAX(lo[c], tt[c]));
                vn[c] = RMIN(vn[c], RMIN(lo[c], tt[c]));
            }
        }
        const int ne = (c_ablate & 2) ? 0 : ni.e1 - ni.e0;
        auto add = [&](int c, real h, int second) {
            if (second) {  // ascending edge order: the reference's sum order (reference.cpp:406-425)
                p[c] += RMAX(0., -h);
                m[c] += RMIN(0., -h);
            } else {
                p[c] += RMAX(0., h);
                m[c] += RMIN(0., h);
            }
        };
        for_edges_cluster<C, EB>(recs[j].edge, 0, min(ne, kRecEdge), a.adf_h, a.LO, a.ttf, z0, L, vx, vn, add);
        if (ne > kRecEdge)
            for_edges_cluster<C, EB>(mp.p_edges, ni.e0 + kRecEdge, ni.e1, a.adf_h, a.LO, a.ttf, z0, L, vx, vn, add);
    }
    real *tvx = lds, *tvn = lds + G * L;
    const int q = j * L + z0;
    if (col) {
#pragma unroll
        for (int c = 0; c < C; c++) {
            tvx[q + c] = vx[c];
            tvn[q + c] = vn[c];
        }
    }
    __syncthreads();
    if (nw == 0) return;
    real ai[C], op[C], om[C];
#pragma unroll
    for (int c = 0; c < C; c++) ai[c] = c < nw ? a.area_inv[ab + c] : 0.;
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
            if (z >= 1 && z < Ln - 1) {
                const size_t bz = b + c;
                const real c0 = RMAX(a.LO[bz - 1], a.ttf[bz - 1]);
                const real c1 = RMAX(a.LO[bz], a.ttf[bz]);
                const real c2 = RMAX(a.LO[bz + 1], a.ttf[bz + 1]);
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
    stv<C>(a.plus + b, op, nw);
    stv<C>(a.minus + b, om, nw);
}

// cluster bound from the staged columns (slot = position in the block's cluster list)
template <int C>
__device__ __forceinline__ void cluster_bound_lds(const RingRef *__restrict__ ring, int r0, int r1,
                                                  const real *smx, const real *smn, int z0, int L,
                                                  real (&vx)[C], real (&vn)[C])
{
    for (int r = r0; r < r1; r++) {
        const RingRef rr = ring[r];
        const int q = rr.node * L + z0;
#pragma unroll
        for (int c = 0; c < C; c++)
            if (z0 + c < rr.lev) {
                vx[c] = RMAX(vx[c], smx[q + c]);
                vn[c] = RMIN(vn[c], smn[q + c]);
            }
    }
}

// Phase 1 (vlimit 1) with the cluster staged: the block's distinct cluster columns (MeshPlanDev
// stage_*) are read once, max/min(LO, ttf) per level go to LDS, and every column's tvert comes from
// LDS -- one round of independent loads instead of a dependent gather batch per cluster member.
// The tvert stencil arrays then reuse the staging area.
template <int C, int EB, int KS>
__global__ __launch_bounds__(1024) void k_p1s(MeshPlanDev mp, P1Args a, int G, float invS, int U)
{
    extern __shared__ real lds[];  // staged max | staged min (U*L each; later tvx | tvn) | NodeRec[G]
    const int L = a.nl - 1, S = L / C;
    const int t = threadIdx.x;
    int tr;
    const int grp = group_tracer(a.tr.n, tr, c_tracer_major & 1);
    const int first = grp * G;
    if (tr) {
        a.ttf += tr * a.tr.node;
        a.LO += tr * a.tr.node;
        a.plus += tr * a.tr.node;
        a.minus += tr * a.tr.node;
        a.adf_v += tr * a.tr.lev;
        a.adf_h += tr * a.tr.edge;
    }
    const int ncol = min(G, a.n_owned - first);
    real *smx = lds, *smn = lds + U * L;
    const NodeRec *recs = stage_records(mp.s_rec, first, ncol, lds + 2 * U * L);
    {
        // every item's index and column loads are issued before any is consumed
        const int u0 = mp.blk_ptr[grp], nitems = (mp.blk_ptr[grp + 1] - u0) * S;
        const int nt = blockDim.x;
        int dst[KS];
        size_t src[KS];
#pragma unroll
        for (int k = 0; k < KS; k++) {
            const int it = t + k * nt;
            int q = 0, sl = 0;
            if (it < nitems) slot_of(it, S, invS, q, sl);
            dst[k] = it < nitems ? q * L + C * sl : -1;
            src[k] = it < nitems ? (size_t)mp.blk_nodes[u0 + q] * L + C * sl : 0;
        }
        real lo[KS][C], tt[KS][C];
#pragma unroll
        for (int k = 0; k < KS; k++)
            if (dst[k] >= 0) {
                ldv<C>(a.LO + src[k], lo[k]);
                ldv<C>(a.ttf + src[k], tt[k]);
            }
#pragma unroll
        for (int k = 0; k < KS; k++)
            if (dst[k] >= 0)
#pragma unroll
                for (int c = 0; c < C; c++) {
                    smx[dst[k] + c] = RMAX(lo[k][c], tt[k][c]);
                    smn[dst[k] + c] = RMIN(lo[k][c], tt[k][c]);
                }
    }
    int j, u;
    slot_of(t, S, invS, j, u);
    const int z0 = C * u;
    const bool col = j < ncol;
    NodeInfo ni{};
    if (col) ni = recs[j].info;
    const int Ln = ni.Ln;
    const int nw = col ? max(0, min(C, Ln - z0)) : 0;
    real vx[C], vn[C], p[C], m[C];
#pragma unroll
    for (int c = 0; c < C; c++) vx[c] = vn[c] = p[c] = m[c] = 0.;
    size_t b = 0, ab = 0;
    if (nw > 0) {
        b = (size_t)ni.n * L + z0;
        ab = (size_t)ni.n * a.nl + z0;
        real v[C + 1];
#pragma unroll
        for (int c = 0; c <= C; c++) v[c] = (c == 0 || c < nw + 1) ? a.adf_v[ab + c] : 0.;
#pragma unroll
        for (int c = 0; c < C; c++) {
            p[c] = RMAX(0., v[c]) + RMAX(0., -v[c + 1]);  // b1-vertical, reference.cpp:393-399
            m[c] = RMIN(0., v[c]) + RMIN(0., -v[c + 1]);
        }
        const int ne = ni.e1 - ni.e0;
        auto add = [&](int c, real h, int second) {
            if (second) {  // ascending edge order: the reference's sum order (reference.cpp:406-425)
                p[c] += RMAX(0., -h);
                m[c] += RMIN(0., -h);
            } else {
                p[c] += RMAX(0., h);
                m[c] += RMIN(0., h);
            }
        };
        for_edges<C, EB>(recs[j].edge, 0, min(ne, kRecEdge), a.adf_h, z0, L, add);
        if (ne > kRecEdge) for_edges<C, EB>(mp.p_edges, ni.e0 + kRecEdge, ni.e1, a.adf_h, z0, L, add);
    }
    __syncthreads();  // staged columns complete
    if (nw > 0) {
#pragma unroll
        for (int c = 0; c < C; c++) {
            const bool dry = z0 + c >= ni.zdry;
            vx[c] = dry ? -a.big : -INFINITY;
            vn[c] = dry ? a.big : INFINITY;
        }
        const int nr = ni.r1 - ni.r0;
        cluster_bound_lds<C>(recs[j].ring, 0, min(nr, kRecRing), smx, smn, z0, L, vx, vn);
        if (nr > kRecRing) cluster_bound_lds<C>(mp.s_ring, ni.r0 + kRecRing, ni.r1, smx, smn, z0, L, vx, vn);
    }
    __syncthreads();  // staging area free: tvert goes there
    real *tvx = lds, *tvn = lds + G * L;
    const int q = j * L + z0;
    if (col) {
#pragma unroll
        for (int c = 0; c < C; c++) {
            tvx[q + c] = vx[c];
            tvn[q + c] = vn[c];
        }
    }
    __syncthreads();
    if (nw == 0) return;
    real lo[C], ai[C], op[C], om[C];
    ldv<C>(a.LO + b, lo);
#pragma unroll
    for (int c = 0; c < C; c++) ai[c] = c < nw ? a.area_inv[ab + c] : 0.;
#pragma unroll
    for (int c = 0; c < C; c++) {
        op[c] = om[c] = 0.;
        const int z = z0 + c;
        if (c >= nw) continue;
        real tm, tn;
        if (z == 0 || z == Ln - 1) {
            tm = tvx[q + c];
            tn = tvn[q + c];
        } else {
            tm = RMAX(RMAX(tvx[q + c - 1], tvx[q + c]), tvx[q + c + 1]);
            tn = RMIN(RMIN(tvn[q + c - 1], tvn[q + c]), tvn[q + c + 1]);
        }
        real flux = p[c] * a.dt * ai[c] + a.eps;  // b2, reference.cpp:432-435
        op[c] = RMIN(1., (tm - lo[c]) / flux);
        flux = m[c] * a.dt * ai[c] - a.eps;
        om[c] = RMIN(1., (tn - lo[c]) / flux);
    }
    stv<C>(a.plus + b, op, nw);
    stv<C>(a.minus + b, om, nw);
}

// Phase 2 with b3-horizontal folded in (b3h + b3v + cv + ch, see launch_p2_fused_b3h).  Each
// endpoint limits its edges' raw fluxes for its own c-horizontal; after the block barrier (every
// raw fct_adf_h read of the block done) one thread per (column, edge) bumps the edge's counter, and
// the endpoint that arrives last -- or the only owned one -- stores the limited column.
template <int C, int KB>
__global__ __launch_bounds__(1024) void k_p2f(MeshPlanDev mp, P2Args a, int G, float invS)
{
    extern __shared__ real lds[];  // NodeRec[G] | writer masks[G]
    const int L = a.nl - 1, S = L / C;
    const int t = threadIdx.x;
    int tr;
    const int first = group_tracer(a.tr.n, tr, c_tracer_major & 4) * G;
    if (tr) {
        a.plus += tr * a.tr.node;
        a.minus += tr * a.tr.node;
        a.ttf += tr * a.tr.node;
        a.LO += tr * a.tr.node;
        a.del_v += tr * a.tr.node;
        a.del_h += tr * a.tr.node;
        a.adf_v += tr * a.tr.lev;
        a.adf_h += tr * a.tr.edge;
        a.edge_cnt += (size_t)tr * mp.n_edges;
    }
    unsigned *wmask = reinterpret_cast<unsigned *>(reinterpret_cast<NodeRec *>(lds) + G);
    if (t < G) wmask[t] = 0u;
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
    const int ne = col ? ni.e1 - ni.e0 : 0;
    real l[C], dv[C], dh[C], pn[C], mn[C];
    size_t b = 0, ab = 0;
    if (na > 0) {
        b = (size_t)ni.n * L + z0;
        ab = (size_t)ni.n * a.nl + z0;
        real pp[C + 2], mm[C + 2], f[C + 1];
        pp[0] = z0 ? a.plus[b - 1] : 0.;
        mm[0] = z0 ? a.minus[b - 1] : 0.;
        ldv<C>(a.plus + b, pn);
        ldv<C>(a.minus + b, mn);
#pragma unroll
        for (int c = 0; c < C; c++) {
            pp[c + 1] = pn[c];
            mm[c + 1] = mn[c];
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
            lim[c] = lim_here ? b3v_factor(z, f[c], pp[c], mm[c], pp[c + 1], mm[c + 1]) * f[c] : f[c];
        }
#pragma unroll
        for (int c = 0; c < C; c++) l[c] = lim[c];
        if (nw > 0) {
            real del_v[C], ttf[C], hn[C], lo[C], hnn[C];
            ldv<C>(a.del_v + b, del_v);
            ldv<C>(a.ttf + b, ttf);
            ldv<C>(a.hnode + b, hn);
            ldv<C>(a.LO + b, lo);
            ldv<C>(a.hnode_new + b, hnn);
            ldv<C>(a.del_h + b, dh);
            real dta[C];
#pragma unroll
            for (int c = 0; c < C; c++) {
                dta[c] = c < nw ? a.dt / a.area[ab + c] : 0.;
                real tv = del_v[c] - ttf[c] * hn[c];  // kernels/fct_ale_c_vertical.cu:9-12 order
                tv = tv + lo[c] * hnn[c];
                dv[c] = tv + (lim[c] - lim[c + 1]) * dta[c];
            }
            auto add = [&](int c, real h, int second, int) {
                dh[c] = second ? dh[c] - h * dta[c] : dh[c] + h * dta[c];  // docs/refactoring.md:311-312
            };
            for_edges_limited<C, KB>(recs[j].edge, 0, min(ne, kRecEdge), a.adf_h, a.plus, a.minus, pn, mn, z0, L, add);
            if (ne > kRecEdge)
                for_edges_limited<C, KB>(mp.p_edges, ni.e0 + kRecEdge, ni.e1, a.adf_h, a.plus, a.minus, pn, mn, z0, L,
                                         add);
        }
    }
    __syncthreads();  // every raw fct_adf_v / fct_adf_h read of the block is done
    if (c_ablate & 8) {  // timing only: static writer, no arrival counters (racy results)
        for (int k = u; k < ne; k += S) {
            const EdgeRef er = k < kRecEdge ? recs[j].edge[k] : mp.p_edges[ni.e0 + k];
            if (!(er.code & 1)) atomicOr(&wmask[j], 1u << k);
        }
    } else {
        for (int k = u; k < ne; k += S) {
            const EdgeRef er = k < kRecEdge ? recs[j].edge[k] : mp.p_edges[ni.e0 + k];
            if (er.other >= a.n_owned || atomicAdd(a.edge_cnt + er.edge, 1) == 1) atomicOr(&wmask[j], 1u << k);
        }
    }
    __syncthreads();
    if (na <= 0) return;
#pragma unroll
    for (int c = 0; c < C; c++)
        if (c < na) a.adf_v[ab + c] = l[c];
    if (nw <= 0) return;
    stv<C>(a.del_v + b, dv, nw);
    stv<C>(a.del_h + b, dh, nw);
    const unsigned mine = wmask[j];
    for (int k = 0; k < ne; k++) {
        if (!((mine >> k) & 1u)) continue;
        const EdgeRef er = k < kRecEdge ? recs[j].edge[k] : mp.p_edges[ni.e0 + k];
        const int lev = er.code >> 1, second = er.code & 1;
        if (z0 >= lev) continue;
        real h[C], po[C], mo[C], out[C];
        const size_t ie = (size_t)er.edge * L + z0;
        ldv<C>(a.adf_h + ie, h);
        ldv<C>(a.plus + (size_t)er.other * L + z0, po);
        ldv<C>(a.minus + (size_t)er.other * L + z0, mo);
#pragma unroll
        for (int c = 0; c < C; c++) {
            const real ae = second ? b3h_factor(h[c], po[c], mo[c], pn[c], mn[c])
                                   : b3h_factor(h[c], pn[c], mn[c], po[c], mo[c]);
            out[c] = ae * h[c];
        }
        stv<C>(a.adf_h + ie, out, min(C, lev - z0));
    }
}

// Chunked phase 2 with the boundary between chunks merged (FESOM2_P2_CHUNK with
// FESOM2_P2_MERGE=1): blocks [0, nb_p2) run the node kernel on chunk c (nb_p2 a multiple of 8, so
// the XCD swizzle applies within each role), the rest b3h on the edges chunk c+1 owns.  The node
// blocks come first in dispatch order; the edge blocks fill the CUs as they drain.
template <int C, int KB, int U>
__global__ __launch_bounds__(1024) void k_p2_b3h_chunk(MeshPlanDev mp, P2Args a, int nb_p2, int G, float invS,
                                                       const int4 *__restrict__ einfo, int n_edges, int Gb,
                                                       float invSb)
{
    extern __shared__ real lds[];  // NodeRec[G] (node blocks)
    const int b = blockIdx.x;
    if (b < nb_p2) {
        const int first = xcd_tile(b, nb_p2) * G;
        if (first >= a.count) return;
        const int ncol = min(G, a.count - first);
        const NodeRec *recs = stage_records(a.nodes, first, ncol, lds);
        p2_node_work<C, KB, true, false>(mp, a, recs, ncol, invS);
    } else {
        const int nb = gridDim.x - nb_p2;
        b3h_groups<C, U, true>(einfo, n_edges, a.nl - 1, Gb, invSb, a.plus, a.minus, a.adf_h, xcd_tile(b - nb_p2, nb));
    }
}

// ---------------------------------------------------------------- persistent phase 2
// b3-horizontal of `count` edges of `ei` by the whole block ((edge, slot) items strided over the
// threads).  The raw flux is read and the limited one written agent-coherently: the node parts of
// other workgroups of this launch read it (write-through stores, no L1 copy; MI355X guide §6 G16).
template <int C>
__device__ __forceinline__ void b3h_block_coherent(const int4 *__restrict__ ei, int count, int L, int S,
                                                   float invS, const real *__restrict__ plus,
                                                   const real *__restrict__ minus, real *adf_h)
{
    constexpr int K = 2;  // items per round: every load of K items issued before any is used
    const int n = count * S;
    for (int base = threadIdx.x; base < n; base += K * (int)blockDim.x) {
        int4 e[K];
        int z0[K];
#pragma unroll
        for (int q = 0; q < K; q++) {
            const int it = base + q * (int)blockDim.x;
            int k = 0, u = 0;
            if (it < n) slot_of(it, S, invS, k, u);
            e[q] = it < n ? ei[k] : make_int4(0, 0, 0, 0);
            z0[q] = C * u;
        }
        real f[K][C], p1[K][C], m1[K][C], p2[K][C], m2[K][C];
#pragma unroll
        for (int q = 0; q < K; q++) {
            if (z0[q] >= e[q].z) continue;
            ldv_coh<C>(adf_h + (size_t)e[q].w * L + z0[q], f[q]);
            ldv<C>(plus + (size_t)e[q].x * L + z0[q], p1[q]);
            ldv<C>(minus + (size_t)e[q].x * L + z0[q], m1[q]);
            ldv<C>(plus + (size_t)e[q].y * L + z0[q], p2[q]);
            ldv<C>(minus + (size_t)e[q].y * L + z0[q], m2[q]);
        }
#pragma unroll
        for (int q = 0; q < K; q++) {
            const int nw = min(C, e[q].z - z0[q]);
#pragma unroll
            for (int c = 0; c < C; c++)
                if (c < nw)
                    __hip_atomic_store(adf_h + (size_t)e[q].w * L + z0[q] + c,
                                       b3h_factor(f[q][c], p1[q][c], m1[q][c], p2[q][c], m2[q][c]) * f[q][c],
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Phase 2 as one persistent launch: workgroup w takes tiles (G positions of the processing order)
// from ticket stream w % 8 in order; per tile it limits the edges the tile owns (its first visited
// endpoint is in the tile), publishes the tile's flag, waits for the flags of the earlier tiles that
// own its other edges, and runs the node kernel on the tile -- the limited fct_adf_h and plus/minus
// it reads were touched moments before, in the caches.  Edge parts never wait and a tile only waits
// for earlier tiles of its own stream, which are already claimed, so every wait ends (spins are
// bounded regardless: state[8] records a timeout).  Edges between streams were limited before the
// launch.
template <int C, int KB>
__global__ __launch_bounds__(1024) void k_p2w(MeshPlanDev mp, P2Args a, int *state, int G, float invS)
{
    extern __shared__ real lds[];  // NodeRec[G] | ticket
    int *sh = reinterpret_cast<int *>(reinterpret_cast<NodeRec *>(lds) + G);
    const int L = a.nl - 1, S = L / C;
    const int x = blockIdx.x % kWfStreams;
    const int tend = mp.wf_stream_first[x + 1];
    int *flags = state + 16;
    for (;;) {
        if (threadIdx.x == 0) sh[0] = mp.wf_stream_first[x] + atomicAdd(state + x, 1);
        __syncthreads();
        const int tile = sh[0];
        if (tile >= tend) return;
        const int e0 = mp.wf_edge_ptr[tile];
        b3h_block_coherent<C>(mp.wf_edges + e0, mp.wf_edge_ptr[tile + 1] - e0, L, S, invS, a.plus, a.minus, a.adf_h);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(flags + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (threadIdx.x < 64) {  // one wave polls the tile's dependencies, relaxed, with back-off
            for (int d = mp.wf_dep_ptr[tile] + (int)threadIdx.x; d < mp.wf_dep_ptr[tile + 1]; d += 64) {
                const int dep = mp.wf_deps[d];
                for (unsigned spins = 0;
                     __hip_atomic_load(flags + dep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0; spins++) {
                    __builtin_amdgcn_s_sleep(2);
                    // bounded: after ~1 s of spinning, or once any wait timed out, give up (the
                    // launch's results are then invalid and state[8] says so)
                    if (spins > (1u << 22) ||
                        ((spins & 1023) == 1023 &&
                         __hip_atomic_load(state + 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
                        __hip_atomic_store(state + 8, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
            }
        }
        __syncthreads();
        const int first = tile * G;
        const int ncol = min(G, a.count - first);
        const NodeRec *recs = stage_records(a.nodes, first, ncol, lds);
        P2Args b = a;
        p2_node_work<C, KB, true, true>(mp, b, recs, ncol, invS);
        __syncthreads();  // LDS and the ticket slot are reused by the next tile
    }
}


// ============================================================================ launchers

hipError_t launch_p1_variant(const MeshPlanDev &mp, const P1Args &a, hipStream_t s, bool *handled)
{
    *handled = true;
    const int L = a.nl - 1, C = levels_per_thread(L), S = L / C, G = group_columns(S);
    const long groups = (long)(a.n_owned + G - 1) / G * a.tr.n;
    // cluster along the edge list (FESOM2_P1_EDGE=1 where the plan verified it; measured equal at
    // EB = 1, slower at EB >= 2: DESIGN.md §3)
    if (mp.edge_cluster && knob("FESOM2_P1_EDGE", 0)) {
        const size_t lds = 2 * (size_t)G * L * sizeof(real) + (size_t)G * sizeof(NodeRec);
        const float invS = 1.0f / (float)S;
        const int EB = knob("FESOM2_P1E_EB", 2);
#define F2A_P1E(CC, EBV)                                                                                        \
        if (a.vlimit == 2) F2A_LAUNCH_GROUPS((k_p1e<2, CC, EBV>), groups, G, S, lds, s, mp, a, G, invS);  \
        if (a.vlimit == 3) F2A_LAUNCH_GROUPS((k_p1e<3, CC, EBV>), groups, G, S, lds, s, mp, a, G, invS);  \
        F2A_LAUNCH_GROUPS((k_p1e<1, CC, EBV>), groups, G, S, lds, s, mp, a, G, invS);
        if (C == 2) {
            if (EB == 1) { F2A_P1E(2, 1) }
            if (EB == 4) { F2A_P1E(2, 4) }
            if (EB == 3) { F2A_P1E(2, 3) }
            F2A_P1E(2, 2)
        }
        F2A_P1E(1, 2)
#undef F2A_P1E
    }
    // staged cluster (FESOM2_P1_STAGE=1; vlimit 1 only; measured slower at G = 8)
    if (a.vlimit == 1 && mp.stage_max > 0 && mp.stage_G == G && knob("FESOM2_P1_STAGE", 0)) {
        const int U = std::max(mp.stage_max, G);
        const size_t lds = 2 * (size_t)U * L * sizeof(real) + (size_t)G * sizeof(NodeRec);
        const float invS = 1.0f / (float)S;
        const int EB = knob("FESOM2_P1S_EB", 2);
        const int KS = (mp.stage_max * S + (int)threads_for(G, S) - 1) / (int)threads_for(G, S);  // items per thread
        if (C == 2 && KS <= 8) {
#define F2A_P1S(EBV, KSV) \
            if (EB == EBV && KS <= KSV) F2A_LAUNCH_GROUPS((k_p1s<2, EBV, KSV>), groups, G, S, lds, s, mp, a, G, invS, U);
            F2A_P1S(2, 2) F2A_P1S(2, 4) F2A_P1S(2, 6) F2A_P1S(2, 8)
            F2A_P1S(4, 2) F2A_P1S(4, 4) F2A_P1S(4, 6) F2A_P1S(4, 8)
#undef F2A_P1S
        }
    }
    *handled = false;
    return hipSuccess;
}

hipError_t launch_p2_fused_b3h(const MeshPlanDev &mp, const P2Args &a, hipStream_t s)
{
    const int L = a.nl - 1, C = levels_per_thread(L), S = L / C, G = group_columns(S);
    const long groups = (long)(a.count + G - 1) / G * a.tr.n;
    const float invS = 1.0f / (float)S;
    const size_t lds = (size_t)G * (sizeof(NodeRec) + sizeof(unsigned));
    const int KB = knob("FESOM2_P2F_BATCH", 2);
    if (C == 2) {
        if (KB == 4) F2A_LAUNCH_GROUPS((k_p2f<2, 4>), groups, G, S, lds, s, mp, a, G, invS);
        if (KB == 1) F2A_LAUNCH_GROUPS((k_p2f<2, 1>), groups, G, S, lds, s, mp, a, G, invS);
        F2A_LAUNCH_GROUPS((k_p2f<2, 2>), groups, G, S, lds, s, mp, a, G, invS);
    }
    F2A_LAUNCH_GROUPS((k_p2f<1, 2>), groups, G, S, lds, s, mp, a, G, invS);
}

hipError_t launch_p2_b3h_chunk(const MeshPlanDev &mp, const P2Args &a, const int4 *einfo, int n_edges, hipStream_t s)
{
    const int L = a.nl - 1, C = levels_per_thread(L), S = L / C, G = group_columns(S);
    if (C != 2 || a.tr.n != 1 || G * S != (int)threads_for(G, S)) return hipErrorInvalidValue;
    const int U = 2;
    const int nb_p2 = ((a.count + G - 1) / G + 7) / 8 * 8;
    const int nb_b3h = (n_edges + U * G - 1) / (U * G);
    const size_t lds = (size_t)G * sizeof(NodeRec);
    const float invS = 1.0f / (float)S;
    init_swizzle();
    if (nb_p2 + nb_b3h > 0)
        hipLaunchKernelGGL((k_p2_b3h_chunk<2, 4, 2>), dim3((unsigned)(nb_p2 + nb_b3h)), dim3(threads_for(G, S)), lds, s, mp,
                           a, nb_p2, G, invS, einfo, n_edges, G, invS);
    return hipGetLastError();
}

hipError_t launch_p2_wavefront(const MeshPlanDev &mp, const P2Args &a, int *state, hipStream_t s)
{
    const int L = a.nl - 1, C = levels_per_thread(L), S = L / C, G = group_columns(S);
    if (G != mp.wf_G || a.tr.n != 1 || a.nodes != mp.node_rec || a.count != mp.n_owned) return hipErrorInvalidValue;
    if (mp.wf_ncross > 0) {
        const hipError_t e = launch_b3h_edges(mp.wf_cross, mp.wf_ncross, a.nl, a.plus, a.minus, a.adf_h, a.tr, s);
        if (e != hipSuccess) return e;
    }
    const float invS = 1.0f / (float)S;
    const size_t lds = (size_t)G * sizeof(NodeRec) + 16;
    const unsigned threads = threads_for(G, S);
    int dev = 0, ncu = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (C == 2)
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)k_p2w<2, 4>, threads, lds);
    else
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)k_p2w<1, 4>, threads, lds);
    long grid = (long)std::max(1, per_cu) * std::max(ncu, 1);
    if (knob("FESOM2_PLAN_STATS", 0)) fprintf(stderr, "fesom2-accelerate: wavefront grid %ld (%d per CU)\n", grid, per_cu);
    grid = std::max<long>(kWfStreams, grid / kWfStreams * kWfStreams);
    init_swizzle();
    if (C == 2)
        hipLaunchKernelGGL((k_p2w<2, 4>), dim3((unsigned)grid), dim3(threads), lds, s, mp, a, state, G, invS);
    else
        hipLaunchKernelGGL((k_p2w<1, 4>), dim3((unsigned)grid), dim3(threads), lds, s, mp, a, state, G, invS);
    return hipGetLastError();
}

}  // namespace f2a
