// f2a_device.hpp -- device helpers and launch utilities shared by the kernel files
// (fct_ale_kernels.hip).
//
// Each kernel file is its own device code object, so the __constant__ switches are per file
// (static) and every file's launchers initialise their own copy (init_swizzle).
#pragma once
#include "f2a_internal.hpp"
#include <algorithm>
#include <cmath>
#include <cstdlib>

namespace f2a {

#define RMAX(a, b) (((a) < (b)) ? (b) : (a))  // std::max(a, b)
#define RMIN(a, b) (((b) < (a)) ? (b) : (a))  // std::min(a, b)

static constexpr int kWave = 64;
static constexpr int kWavesPerBlock = 4;
static constexpr int kBlock = kWave * kWavesPerBlock;

// Bijective XCD-aware swizzle: blocks b and b+8 share an XCD (round-robin dispatch), so hand each
// residue class a contiguous range of tiles.  Speed only, never correctness.
// The switches below are compile-time constants in the product build (their measured defaults) and
// __constant__ knobs only in the tuning build (F2A_TUNING, `make tuning`):
//   c_xcd_swizzle   FESOM2_XCD=0 disables the swizzle (A/B measurements)
//   c_ablate        FESOM2_ABLATE, timing-only experiments (results are wrong): bit 0 skips the cluster
//                   gathers of phase 1, bit 1 its edge gathers, bit 2 the edge gathers of phase 2;
//                   p1v: bit 3 the second fct_adf_v load (the level below the pair), bit 4 the
//                   vertical tail's loads (del_ttf_advvert, hnode, hnode_new, area), bit 5 the union DMA; bit 6
//                   packed b3h's plus/minus gathers
//   c_tracer_major  FESOM2_TRACER_MAJOR bits (batched tracers; 1 p1, 2 b3h, 4 p2): tracer-slowest tile
//                   order; measured: b3h tracer-slowest, p1/p2 tracer-fastest
//   c_tile_rev      FESOM2_TILE_REV bits (1 p1, 2 b3h, 4 p2): the kernel walks each XCD's tile range
//                   backwards, so it starts on the data the previous kernel touched last (still in the
//                   Infinity Cache); the product takes the direction per call (Tracers::order)
//   c_tracer_group  FESOM2_TRACER_GROUP = g (batched tracers, tracer-fastest kernels): tiles run in
//                   groups of g tracers -- every column group for tracers 0..g-1, then g..2g-1 -- so a
//                   column's reuse by the next patch row comes g, not ntracers, tiles later per column
#if F2A_TUNING
static __constant__ int c_xcd_swizzle = 1;
static __constant__ int c_ablate = 0;
static __constant__ int c_tracer_major = 2;
static __constant__ int c_tile_rev = 0;
static __constant__ int c_tracer_group = 0;
#else
static constexpr int c_xcd_swizzle = 1;
static constexpr int c_ablate = 0;
static constexpr int c_tracer_major = 2;
static constexpr int c_tile_rev = 0;
static constexpr int c_tracer_group = 0;
#endif

__device__ __forceinline__ int xcd_tile(int b, int G)
{
    if (!c_xcd_swizzle) return b;
    const int q = G >> 3, r = G & 7, x = b & 7, k = b >> 3;
    return x * q + (x < r ? x : r) + k;
}

// the same ranges, each walked from its end (bijective: XCD x has q + (x < r) tiles)
__device__ __forceinline__ int xcd_tile_rev(int b, int G)
{
    if (!c_xcd_swizzle) return G - 1 - b;
    const int q = G >> 3, r = G & 7, x = b & 7, k = b >> 3;
    const int len = q + (x < r ? 1 : 0);
    return x * q + (x < r ? x : r) + (len - 1 - k);
}

// the tuning build's knobs of the __constant__ switches above (the product keeps the defaults), read
// at every launch and copied to the device when they change -- so an in-process A/B
// (tools/ab_inproc.py) can switch them between bursts
static void init_swizzle()
{
#if F2A_TUNING
    static int last[5] = {1, 2, 0, 0, 0};  // the __constant__ initialisers
    const int v[5] = {knob("FESOM2_XCD", 1) == 0 ? 0 : 1, knob("FESOM2_TRACER_MAJOR", 2), knob("FESOM2_ABLATE", 0),
                      knob("FESOM2_TILE_REV", 0), knob("FESOM2_TRACER_GROUP", 0)};
    const void *sym[5] = {(const void *)&c_xcd_swizzle, (const void *)&c_tracer_major, (const void *)&c_ablate,
                          (const void *)&c_tile_rev, (const void *)&c_tracer_group};
    for (int k = 0; k < 5; k++)
        if (v[k] != last[k]) {
            (void)hipMemcpyToSymbol(sym[k], &v[k], sizeof v[k]);
            last[k] = v[k];
        }
#endif
}

__device__ __forceinline__ int wave_item()
{
    const int t = xcd_tile(blockIdx.x, gridDim.x);
    return __builtin_amdgcn_readfirstlane(t * kWavesPerBlock + (int)(threadIdx.x >> 6));
}

__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

static inline unsigned grid_for(long items)
{
    return (unsigned)((items + kWavesPerBlock - 1) / kWavesPerBlock);
}

// b3-vertical limiter factor of interface z (docs/refactoring.md:205-231).
__device__ __forceinline__ real b3v_factor(int z, real flux, real p_zm1, real m_zm1, real p_z,
                                           real m_z)
{
    real ae = 1.0;
    if (z == 0) {
        ae = (flux >= 0.0) ? RMIN(ae, p_z) : RMIN(ae, m_z);
    } else if (flux >= 0.0) {
        ae = RMIN(ae, m_zm1);
        ae = RMIN(ae, p_z);
    } else {
        ae = RMIN(ae, p_zm1);
        ae = RMIN(ae, m_z);
    }
    return ae;
}

// b3-horizontal factor (docs/refactoring.md:246-257).
__device__ __forceinline__ real b3h_factor(real flux, real p1, real m1, real p2, real m2)
{
    real ae = 1.0;
    if (flux >= 0.0) {
        ae = RMIN(ae, p1);
        ae = RMIN(ae, m2);
    } else {
        ae = RMIN(ae, m1);
        ae = RMIN(ae, p2);
    }
    return ae;
}

// ============================================================================ fused kernels
//
// C levels per thread (C = 2: ttf/LO/adf_h/plus/minus/del_* are read and written as 16-byte pairs;
// the stride-nl arrays -- fct_adf_v, area, area_inv -- and odd-L columns start at 8-byte alignment,
// which a 16-byte access tolerates on gfx950 (f2a_d2u below); for odd L the last slot of a column
// holds one level, see ldo).  A block owns G whole columns (node columns for phases
// 1/2, edge columns for b3h) taken in the plan's processing order; thread t is the level pair
// z0 = C*(t % (L/C)) of column t / (L/C), and the block has G*L/C threads rounded up to the wave
// size (L = 80, C = 2, G = 8: 320 threads, 5 full waves).  A column group completes within one chain
// of memory latencies and the XCD's in-flight window stays a few hundred columns wide, which is
// what lets neighbouring columns' gathers hit its L2.  Columns never straddle blocks, so the LDS
// stencil of phase 1 and the in-place fct_adf_v update of phase 2 only need block barriers.


// t -> (column j, slot u) for t < G*S (S slots per column), exact: the float quotient stays far
// from an integer
__device__ __forceinline__ void slot_of(int t, int S, float invS, int &j, int &u)
{
    j = (int)(((float)t + 0.5f) * invS);
    u = t - j * S;
}

__device__ __forceinline__ int block_tile() { return xcd_tile(blockIdx.x, gridDim.x); }

// tile -> (column group, tracer): tracer fastest (the ntr blocks of a group share the XCD's L2
// for the records and the mesh fields) or, with `major`, tracer slowest (each tracer's gathers
// keep the L2 to themselves)
// (tuning: FESOM2_TRACER_GROUP = g > 1 tiles g tracers at a time -- every column group of tracers
// 0..g-1 first, then the next g; measured neutral at 6 x 127k x 47 and 6 x 1.2M x 80)
__device__ __forceinline__ int group_tracer(int ntr, int &tr, bool major = false, bool rev = false)
{
    const int t = rev ? xcd_tile_rev(blockIdx.x, gridDim.x) : block_tile();
    if (ntr == 1) {
        tr = 0;
        return t;
    }
    if (major) {
        const int groups = gridDim.x / ntr;
        tr = t / groups;
        return t - tr * groups;
    }
    const int gs = c_tracer_group;
    if (gs > 1 && gs < ntr && ntr % gs == 0) {
        const int span = gridDim.x / ntr * gs;  // tiles of one tracer group
        const int tg = t / span, rem = t - tg * span, g = rem / gs;
        tr = tg * gs + (rem - g * gs);
        return g;
    }
    const int g = t / ntr;
    tr = t - g * ntr;
    return g;
}


// 16-byte pair of levels.  Columns of odd-L arrays and of the stride-nl arrays start at 8-byte
// alignment only; a 16-byte load/store at 8-byte alignment is legal on gfx950 (the compiler emits
// the same global_load_dwordx4 / global_store_dwordx4 it emits for 16-byte alignment).
typedef double f2a_d2u __attribute__((ext_vector_type(2), aligned(8)));

// C consecutive levels; C even reads 16-byte pairs (p 8-byte aligned)
template <int C>
__device__ __forceinline__ void ldv(const real *__restrict__ p, real (&v)[C])
{
    if constexpr (C == 1) {
        v[0] = p[0];
    } else {
#pragma unroll
        for (int c = 0; c < C; c += 2) {
            const f2a_d2u t = *reinterpret_cast<const f2a_d2u *>(p + c);
            v[c] = t.x;
            v[c + 1] = t.y;
        }
    }
}

// store the first `n` (1..C) values
template <int C>
__device__ __forceinline__ void stv(real *__restrict__ p, const real (&v)[C], int n)
{
    if constexpr (C == 1) {
        p[0] = v[0];
    } else {
#pragma unroll
        for (int c = 0; c < C; c += 2) {
            if (c + 2 <= n) {
                f2a_d2u t;
                t.x = v[c];
                t.y = v[c + 1];
                *reinterpret_cast<f2a_d2u *>(p + c) = t;
            } else if (c < n) {
                p[c] = v[c];
            }
        }
    }
}

// Single-use streams (a column nobody else reads in the same kernel) can bypass the L2 with
// non-temporal loads/stores, leaving it to the gathered columns.
typedef f2a_d2u f2a_d2;
template <int C, bool NT>
__device__ __forceinline__ void ldv_s(const real *__restrict__ p, real (&v)[C])
{
    if constexpr (NT && C % 2 == 0) {
#pragma unroll
        for (int c = 0; c < C; c += 2) {
            const f2a_d2 t = __builtin_nontemporal_load(reinterpret_cast<const f2a_d2 *>(p + c));
            v[c] = t.x;
            v[c + 1] = t.y;
        }
    } else if constexpr (NT && C == 1) {
        v[0] = __builtin_nontemporal_load(p);
    } else {
        ldv<C>(p, v);
    }
}
template <int C, bool NT>
__device__ __forceinline__ void stv_s(real *__restrict__ p, const real (&v)[C], int n)
{
    if constexpr (NT && C % 2 == 0) {
#pragma unroll
        for (int c = 0; c < C; c += 2) {
            if (c + 2 <= n) {
                f2a_d2 t;
                t.x = v[c];
                t.y = v[c + 1];
                __builtin_nontemporal_store(t, reinterpret_cast<f2a_d2 *>(p + c));
            } else if (c < n) {
                p[c] = v[c];
            }
        }
    } else if constexpr (NT && C == 1) {
        __builtin_nontemporal_store(v[0], p);
    } else {
        stv<C>(p, v, n);
    }
}

// Odd L in pairs (C = 2, S = (L+1)/2 slots per column): the last slot of a column holds the one
// level z0 = L-1 (`last1`).  Its pair load reads that level and the next one -- the next column's
// first level, or for the last column of an array the allocation's pad (kAllocPad) -- and the
// second value is never used: every consumer guards the levels beyond the column (stores write
// `nw` levels, gathers test z0 + c < lev, the LDS images skip it).  Round 2 shifted the last pair
// one level back instead (`p - 1`, then a select per value): the selects and the shifted addresses
// cost 8-10 VGPRs, i.e. 6-7 instead of 8 waves/SIMD for the odd-L p1v.  `last1` stays in the
// signatures for the callers' guards.
template <int C, bool ODD>
__device__ __forceinline__ void ldo(const real *__restrict__ p, real (&v)[C], bool last1)
{
    (void)last1;
    ldv<C>(p, v);
}
template <int C, bool ODD>
__device__ __forceinline__ void ldo_pre(const real *__restrict__ p, real (&v)[C], bool last1)
{
    (void)last1;
    ldv<C>(p, v);
}
template <int C, bool NT, bool ODD>
__device__ __forceinline__ void ldo_s_pre(const real *__restrict__ p, real (&v)[C], bool last1)
{
    (void)last1;
    ldv_s<C, NT>(p, v);
}
template <int C, bool NT, bool ODD>
__device__ __forceinline__ void ldo_s(const real *__restrict__ p, real (&v)[C], bool last1)
{
    (void)last1;
    ldv_s<C, NT>(p, v);
}

// Columns of the stride-nl arrays (fct_adf_v, area, area_inv) start at 8-byte alignment only; a
// 16-byte load at 8-byte alignment (legal on gfx950: the compiler emits global_load_dwordx4 for
// it) halves their load instructions.  Both levels of a pair lie inside the column (z0 + 1 <= L <
// nl), so the second is loaded even when only the first is wet; it is then replaced by `fill`.
template <int C, bool PAIR>
__device__ __forceinline__ void ld_nl(const real *__restrict__ p, int nw, real (&v)[C], real fill)
{
    if constexpr (PAIR && C == 2) {
        const f2a_d2u t = *reinterpret_cast<const f2a_d2u *>(p);
        v[0] = t.x;
        v[1] = nw >= 2 ? t.y : fill;
    } else {
#pragma unroll
        for (int c = 0; c < C; c++) v[c] = c < nw ? p[c] : fill;
    }
}

template <bool NT>
__device__ __forceinline__ real ld1_s(const real *__restrict__ p)
{
    if constexpr (NT) return __builtin_nontemporal_load(p);
    return *p;
}
template <bool NT>
__device__ __forceinline__ void st1_s(real *__restrict__ p, real v)
{
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// the level count an EdgeRef::code carries (bits 1..11; bit 0 = second endpoint, bits 12 and up the
// LDS-stash slot of a block-internal edge, see kStashShift): every decode goes through here
__device__ __forceinline__ int edge_lev(int code) { return (code >> 1) & kLevMask; }

// tvert(n, z): max/min over the elements around n of UV_rhs(e, z) (reference.cpp:358-378), taken
// straight from ttf/LO over the node's cluster (a1 + a2 + the cluster part of a3, see RingRef).
// (vx, vn must be initialised by the caller: -/+bignumber where an adjacent element is dry, else
// -/+infinity)
template <int C, int kBatch, bool ODD = false>
__device__ __forceinline__ void cluster_bound(const RingRef *__restrict__ ring, int r0, int r1,
                                              const real *__restrict__ LO,
                                              const real *__restrict__ ttf, int z0, int L,
                                              real (&vx)[C], real (&vn)[C], bool last1 = false)
{
    const int zl = z0;  // odd L: the last pair reads one level past the column (ldo)
    for (int r = r0; r < r1; r += kBatch) {
        size_t idx[kBatch];
        int lev[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            const RingRef rr = (r + k < r1) ? ring[r + k] : RingRef{0, 0};
            idx[k] = (size_t)rr.node * L + zl;
            lev[k] = rr.lev & kLevMask;  // (above it: the p1v block's union slot, MeshPlanDev::cu_ptr)
        }
        real lo[kBatch][C], tt[kBatch][C];
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            if (z0 < lev[k]) {
                ldo_pre<C, ODD>(LO + idx[k], lo[k], last1);
                ldo_pre<C, ODD>(ttf + idx[k], tt[k], last1);
            } else {
#pragma unroll
                for (int c = 0; c < C; c++) lo[k][c] = tt[k][c] = 0.;
            }
        }
#pragma unroll
        for (int k = 0; k < kBatch; k++)
#pragma unroll
            for (int c = 0; c < C; c++)
                if (z0 + c < lev[k]) {
                    vx[c] = RMAX(vx[c], RMAX(lo[k][c], tt[k][c]));
                    vn[c] = RMIN(vn[c], RMIN(lo[k][c], tt[k][c]));
                }
    }
}

// Gather the fct_adf_h levels z0..z0+C-1 of a node's edges (CSR slice [e0, e1), ascending edge
// order) and hand each (value, second-endpoint flag) to `f(c, h, second)` in that order.
template <int C, int kBatch, bool ODD = false, class F>
__device__ __forceinline__ void for_edges(const EdgeRef *__restrict__ edges, int e0, int e1,
                                          const real *__restrict__ adf_h, int z0, int L, F &&f,
                                          bool last1 = false, real *stash = nullptr)
{
    const int zl = z0;  // odd L: the last pair reads one level past the column (ldo)
    for (int k0 = e0; k0 < e1; k0 += kBatch) {
        size_t idx[kBatch];
        int code[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            const EdgeRef er = (k0 + k < e1) ? edges[k0 + k] : EdgeRef{0, 0, 0};
            idx[k] = (size_t)er.edge * L + zl;
            code[k] = er.code;
        }
        real h[kBatch][C];
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            if (z0 < edge_lev(code[k])) {
                ldo_pre<C, ODD>(adf_h + idx[k], h[k], last1);
            } else {
#pragma unroll
                for (int c = 0; c < C; c++) h[k][c] = 0.;
            }
        }
        if (stash) {  // (large partitions; OPT & 256 of k_p1) the block-internal edges' raw flux into LDS
#pragma unroll
            for (int k = 0; k < kBatch; k++) {
                const int sl = code[k] >> kStashShift;
                if (!sl) continue;
                real *sp = stash + (sl - 1) * L + z0;
                const int lv = edge_lev(code[k]);
                if constexpr (C == 2) {  // one 16-B LDS store for a full pair (8-B aligned: ds_write2)
                    if (z0 + 1 < lv) {
                        f2a_d2u t;
                        t.x = h[k][0];
                        t.y = h[k][1];
                        *reinterpret_cast<f2a_d2u *>(sp) = t;
                    } else if (z0 < lv) {
                        sp[0] = h[k][0];
                    }
                } else {
#pragma unroll
                    for (int c = 0; c < C; c++)
                        if (z0 + c < lv) sp[c] = h[k][c];
                }
            }
        }
#pragma unroll
        for (int k = 0; k < kBatch; k++)
#pragma unroll
            for (int c = 0; c < C; c++)
                if (z0 + c < edge_lev(code[k])) f(c, h[k][c], code[k] & 1);
    }
}

// Edge gathers with the b3-horizontal limiter applied in-thread: for kBatch edges at a time the raw
// flux and the other endpoint's plus/minus are loaded, then f(c, limited flux, second) runs in
// ascending edge order.  (pn, mn: this node's plus/minus at the thread's levels.)
template <int C, int kBatch, bool ODD = false, class F>
__device__ __forceinline__ void for_edges_limited(const EdgeRef *__restrict__ edges, int e0, int e1,
                                                  const real *__restrict__ adf_h,
                                                  const real *__restrict__ plus,
                                                  const real *__restrict__ minus, const real (&pn)[C],
                                                  const real (&mn)[C], int z0, int L, F &&f, bool last1 = false)
{
    for (int k0 = e0; k0 < e1; k0 += kBatch) {
        EdgeRef er[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; k++) er[k] = (k0 + k < e1) ? edges[k0 + k] : EdgeRef{0, 0, 0};
        real h[kBatch][C], po[kBatch][C], mo[kBatch][C];
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            if (z0 < edge_lev(er[k].code)) {
                ldo<C, ODD>(adf_h + (size_t)er[k].edge * L + z0, h[k], last1);
                ldo<C, ODD>(plus + (size_t)er[k].other * L + z0, po[k], last1);
                ldo<C, ODD>(minus + (size_t)er[k].other * L + z0, mo[k], last1);
            }
        }
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            const int lev = edge_lev(er[k].code), second = er[k].code & 1;
#pragma unroll
            for (int c = 0; c < C; c++) {
                if (z0 + c >= lev) continue;
                // docs/refactoring.md:246-257 with (n1, n2) = (other, this) when second
                const real ae = second ? b3h_factor(h[k][c], po[k][c], mo[k][c], pn[c], mn[c])
                                       : b3h_factor(h[k][c], pn[c], mn[c], po[k][c], mo[k][c]);
                f(c, ae * h[k][c], second, k0 + k);
            }
        }
    }
}

// Stage the block's NodeRec records (one coalesced 16-byte-per-thread sweep) into LDS after
// `lds_base`; ends with a block barrier.
__device__ __forceinline__ const NodeRec *stage_records(const NodeRec *__restrict__ recs, int first, int ncol,
                                                        real *lds_base)
{
    NodeRec *r = reinterpret_cast<NodeRec *>(lds_base);
    const int4 *src = reinterpret_cast<const int4 *>(recs + first);
    int4 *dst = reinterpret_cast<int4 *>(r);
    constexpr int kChunks = sizeof(NodeRec) / sizeof(int4);
    for (int i = threadIdx.x; i < ncol * kChunks; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
    return r;
}

// Same, U consecutive edge groups per block: every einfo load of the U groups is issued, then every
// data load, so a thread keeps U x 5 loads in flight instead of 5 (memory-level parallelism), and
// the grid has U times fewer blocks.  NT: fct_adf_h streamed with non-temporal loads/stores so the
// gathered plus/minus columns keep the L2.
// U edge groups starting at group `ug` (relative to einfo) of one tracer.
template <int C, int U, bool NT, bool ODD = false>
__device__ __forceinline__ void b3h_groups(const int4 *__restrict__ einfo, int n_edges, int L, int G, float invS,
                                           const real *__restrict__ plus, const real *__restrict__ minus,
                                           real *__restrict__ adf_h, int ug)
{
    int j, u;
    slot_of(threadIdx.x, (L + C - 1) / C, invS, j, u);
    if (j >= G) return;
    const int z0 = C * u;
    const bool last1 = ODD && z0 + 1 == L;
    const int k0 = ug * U * G + j;
    int4 ei[U];
#pragma unroll
    for (int q = 0; q < U; q++) {
        const int k = k0 + q * G;
        ei[q] = k < n_edges ? einfo[k] : make_int4(0, 0, 0, 0);
    }
    real f[U][C], p1[U][C], m1[U][C], p2[U][C], m2[U][C];
#pragma unroll
    for (int q = 0; q < U; q++) {
        if (z0 < ei[q].z) {
            ldo_s<C, NT, ODD>(adf_h + (size_t)ei[q].w * L + z0, f[q], last1);
            const size_t i1 = (size_t)ei[q].x * L + z0, i2 = (size_t)ei[q].y * L + z0;
            ldo<C, ODD>(plus + i1, p1[q], last1);
            ldo<C, ODD>(minus + i1, m1[q], last1);
            ldo<C, ODD>(plus + i2, p2[q], last1);
            ldo<C, ODD>(minus + i2, m2[q], last1);
        }
    }
#pragma unroll
    for (int q = 0; q < U; q++) {
        const int nw = min(C, ei[q].z - z0);
        if (nw <= 0) continue;
        real out[C];
#pragma unroll
        for (int c = 0; c < C; c++) out[c] = b3h_factor(f[q][c], p1[q][c], m1[q][c], p2[q][c], m2[q][c]) * f[q][c];
        stv_s<C, NT>(adf_h + (size_t)ei[q].w * L + z0, out, nw);
    }
}

// Phase 2, nodes: b3v + cv + ch, G node columns per block.  fct_adf_h already holds the b3-limited
// fluxes (k_b3h_g ran first, as in docs/refactoring.md:237-314).  The limited vertical flux of the
// interface below a thread's levels is recomputed in-thread from plus/minus (the bottom interface
// nlev-1 is never limited); the barrier orders every raw fct_adf_v read of the block before its
// writes.
// The node work of phase 2 for the block's G columns (records staged): see k_p2.
template <int C, int KB, bool NT>
__device__ __forceinline__ void p2_node_work(const MeshPlanDev &mp, P2Args &a, const NodeRec *recs, int ncol,
                                             float invS)
{
    const int L = a.nl - 1, S = L / C;
    const int t = threadIdx.x;
    int j, u;
    slot_of(t, S, invS, j, u);
    const int z0 = C * u;
    const bool col = j < ncol;
    NodeInfo ni{};
    if (col) ni = recs[j].info;
    const int Ln = ni.Ln;
    const int top = Ln > 1 ? Ln : 1;                   // the Fortran always limits nz = 1
    const int na = col ? max(0, min(C, top - z0)) : 0;  // cells whose adf_v is limited
    const int nw = col ? max(0, min(C, Ln - z0)) : 0;   // wet cells (c-step)
    real l[C], dv[C], dh[C];
    size_t b = 0, ab = 0;
    if (na > 0) {
        b = (size_t)ni.n * L + z0;
        ab = (size_t)ni.n * a.nl + z0;
        // plus/minus at z0-1 .. z0+C, fct_adf_v at z0 .. z0+C
        real pp[C + 2], mm[C + 2], f[C + 1];
        pp[0] = z0 ? a.plus[b - 1] : 0.;
        mm[0] = z0 ? a.minus[b - 1] : 0.;
        {
            real tp[C], tmn[C];
            ldv_s<C, NT>(a.plus + b, tp);
            ldv_s<C, NT>(a.minus + b, tmn);
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
        real lim[C + 1];  // limited adf_v at z0 .. z0+C (raw where not limited)
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
            ldv_s<C, NT>(a.del_v + b, del_v);
            ldv_s<C, NT>(a.ttf + b, ttf);
            ldv_s<C, NT>(a.hnode + b, hn);
            ldv_s<C, NT>(a.LO + b, lo);
            ldv_s<C, NT>(a.hnode_new + b, hnn);
            ldv_s<C, NT>(a.del_h + b, dh);
            real dta[C];
#pragma unroll
            for (int c = 0; c < C; c++) {
                dta[c] = c < nw ? a.dt / ld1_s<NT>(a.area + ab + c) : 0.;
                real tv = del_v[c] - ttf[c] * hn[c];  // kernels/fct_ale_c_vertical.cu:9-12 order
                tv = tv + lo[c] * hnn[c];
                dv[c] = tv + (lim[c] - lim[c + 1]) * dta[c];
            }
            const int ne = (c_ablate & 4) ? 0 : ni.e1 - ni.e0;
            auto add = [&](int c, real h, int second) {
                dh[c] = second ? dh[c] - h * dta[c] : dh[c] + h * dta[c];  // docs/refactoring.md:311-312
            };
            for_edges<C, KB>(recs[j].edge, 0, min(ne, kRecEdge), a.adf_h, z0, L, add);
            if (ne > kRecEdge) for_edges<C, KB>(mp.p_edges, ni.e0 + kRecEdge, ni.e1, a.adf_h, z0, L, add);
        }
    }
    __syncthreads();
    if (na <= 0) return;
#pragma unroll
    for (int c = 0; c < C; c++)
        if (c < na) st1_s<NT>(a.adf_v + ab + c, l[c]);
    if (nw <= 0) return;
    stv_s<C, NT>(a.del_v + b, dv, nw);
    stv_s<C, NT>(a.del_h + b, dh, nw);
}

// ---- host-side launch utilities
static inline unsigned threads_for(int G, int S) { return (unsigned)(((G * S + kWave - 1) / kWave) * kWave); }

// columns per block of a plan's column-group kernels for S slots per column: the plan's explicit
// count (MeshPlanDev::gcols, validated against the widest column shape) or group_columns' natural
// one times 2^gshift
static inline int plan_columns(int S, const MeshPlanDev &mp) { return mp.gcols > 0 ? mp.gcols : group_columns(S, mp.gshift); }

// odd L in level pairs (the last slot of a column holds one level; FESOM2_ODD_PAIR=0 in the tuning
// build: one level per thread)
static inline bool odd_pairs(int L) { return L % 2 == 1 && L >= 3 && knob("FESOM2_ODD_PAIR", 1) != 0; }

static inline int levels_per_thread(int L)
{
    if (knob("FESOM2_CPT", 0) == 1) return 1;  // one level per thread (tuning build only)
    return (L % 2 == 0) ? 2 : 1;
}

#define F2A_LAUNCH_GROUPS(kernel, groups, G, L, lds_bytes, s, ...)                                       \
    do {                                                                                                \
        init_swizzle();                                                                                 \
        if ((groups) > 0)                                                                               \
            hipLaunchKernelGGL(kernel, dim3((unsigned)(groups)), dim3(threads_for(G, L)), (lds_bytes), \
                               (s), __VA_ARGS__);                                                       \
        return hipGetLastError();                                                                       \
    } while (0)

}  // namespace f2a
