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
#include "f2a_internal.hpp"
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
__constant__ int c_xcd_swizzle = 1;  // FESOM2_XCD=0 disables (A/B measurements)
// FESOM2_ABLATE (timing-only builds of an experiment, results are wrong): bit 0 skips the cluster
// gathers of phase 1, bit 1 its edge gathers, bit 2 the edge gathers of phase 2, bit 3 the arrival
// counters of the fused b3h.
__constant__ int c_ablate = 0;
// FESOM2_TRACER_MAJOR bits (batched tracers; 1 p1, 2 b3h, 4 p2): tracer-slowest tile order
__constant__ int c_tracer_major = 2;  // measured: b3h tracer-slowest, p1/p2 tracer-fastest

__device__ __forceinline__ int xcd_tile(int b, int G)
{
    if (!c_xcd_swizzle) return b;
    const int q = G >> 3, r = G & 7, x = b & 7, k = b >> 3;
    return x * q + (x < r ? x : r) + k;
}

static void init_swizzle()
{
    static bool done = false;
    if (done) return;
    done = true;
    const char *e = getenv("FESOM2_XCD");
    if (e && atoi(e) == 0) {
        const int zero = 0;
        (void)hipMemcpyToSymbol(HIP_SYMBOL(c_xcd_swizzle), &zero, sizeof zero);
    }
    const char *tm = getenv("FESOM2_TRACER_MAJOR");
    if (tm) {
        const int v = atoi(tm);
        (void)hipMemcpyToSymbol(HIP_SYMBOL(c_tracer_major), &v, sizeof v);
    }
    const char *ab = getenv("FESOM2_ABLATE");
    if (ab && atoi(ab)) {
        const int v = atoi(ab);
        (void)hipMemcpyToSymbol(HIP_SYMBOL(c_ablate), &v, sizeof v);
    }
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
    for (int k = e0; k < e1; k++) lmax = max(lmax, mp.edges[k].code >> 1);
    const size_t b = (size_t)n * L;
    for (int z = lane; z < lmax; z += kWave) {
        real p = plus[b + z], m = minus[b + z];
        for (int k = e0; k < e1; k++) {
            const EdgeRef er = mp.edges[k];
            if (z < (er.code >> 1)) {
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
    for (int k = e0; k < e1; k++) lmax = max(lmax, mp.edges[k].code >> 1);
    const size_t b = (size_t)n * L, a = (size_t)n * (L + 1);
    for (int z = lane; z < lmax; z += kWave) {
        const real dta = dt / area[a + z];
        real d = del_h[b + z];
        for (int k = e0; k < e1; k++) {
            const EdgeRef er = mp.edges[k];
            if (z < (er.code >> 1)) {
                const real h = adf_h[(size_t)er.edge * L + z];
                d = (er.code & 1) ? d - h * dta : d + h * dta;
            }
        }
        del_h[b + z] = d;
    }
}

// ============================================================================ fused kernels
//
// C levels per thread (C = 2 when L is even: ttf/LO/adf_h/plus/minus/del_* are then read and written
// as 16-byte pairs; arrays of stride nl = L+1 -- fct_adf_v, area, area_inv -- stay 8-byte because
// their columns alternate 16-byte alignment).  A block owns G whole columns (node columns for phases
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
__device__ __forceinline__ int group_tracer(int ntr, int &tr, bool major = false)
{
    const int t = block_tile();
    if (ntr == 1) {
        tr = 0;
        return t;
    }
    if (major) {
        const int groups = gridDim.x / ntr;
        tr = t / groups;
        return t - tr * groups;
    }
    const int g = t / ntr;
    tr = t - g * ntr;
    return g;
}


// C consecutive levels; C even reads 16-byte pairs (p 16-byte aligned)
template <int C>
__device__ __forceinline__ void ldv(const real *__restrict__ p, real (&v)[C])
{
    if constexpr (C == 1) {
        v[0] = p[0];
    } else {
#pragma unroll
        for (int c = 0; c < C; c += 2) {
            const double2 t = *reinterpret_cast<const double2 *>(p + c);
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
            if (c + 2 <= n)
                *reinterpret_cast<double2 *>(p + c) = make_double2(v[c], v[c + 1]);
            else if (c < n)
                p[c] = v[c];
        }
    }
}

// Single-use streams (a column nobody else reads in the same kernel) can bypass the L2 with
// non-temporal loads/stores, leaving it to the gathered columns.
typedef double f2a_d2 __attribute__((ext_vector_type(2)));
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

// tvert(n, z): max/min over the elements around n of UV_rhs(e, z) (reference.cpp:358-378), taken
// straight from ttf/LO over the node's cluster (a1 + a2 + the cluster part of a3, see RingRef).
// (vx, vn must be initialised by the caller: -/+bignumber where an adjacent element is dry, else
// -/+infinity)
template <int C, int kBatch>
__device__ __forceinline__ void cluster_bound(const RingRef *__restrict__ ring, int r0, int r1,
                                              const real *__restrict__ LO,
                                              const real *__restrict__ ttf, int z0, int L,
                                              real (&vx)[C], real (&vn)[C])
{
    for (int r = r0; r < r1; r += kBatch) {
        size_t idx[kBatch];
        int lev[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            const RingRef rr = (r + k < r1) ? ring[r + k] : RingRef{0, 0};
            idx[k] = (size_t)rr.node * L + z0;
            lev[k] = rr.lev;
        }
        real lo[kBatch][C], tt[kBatch][C];
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            if (z0 < lev[k]) {
                ldv<C>(LO + idx[k], lo[k]);
                ldv<C>(ttf + idx[k], tt[k]);
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
// agent-coherent loads (read-only data another workgroup of this launch published: no L1 hit)
template <int C>
__device__ __forceinline__ void ldv_coh(const real *p, real (&v)[C])
{
#pragma unroll
    for (int c = 0; c < C; c++) v[c] = __hip_atomic_load(p + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int C, int kBatch, bool COH = false, class F>
__device__ __forceinline__ void for_edges(const EdgeRef *__restrict__ edges, int e0, int e1,
                                          const real *__restrict__ adf_h, int z0, int L, F &&f)
{
    for (int k0 = e0; k0 < e1; k0 += kBatch) {
        size_t idx[kBatch];
        int code[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            const EdgeRef er = (k0 + k < e1) ? edges[k0 + k] : EdgeRef{0, 0, 0};
            idx[k] = (size_t)er.edge * L + z0;
            code[k] = er.code;
        }
        real h[kBatch][C];
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            if (z0 < (code[k] >> 1)) {
                if constexpr (COH)
                    ldv_coh<C>(adf_h + idx[k], h[k]);
                else
                    ldv<C>(adf_h + idx[k], h[k]);
            } else {
#pragma unroll
                for (int c = 0; c < C; c++) h[k][c] = 0.;
            }
        }
#pragma unroll
        for (int k = 0; k < kBatch; k++)
#pragma unroll
            for (int c = 0; c < C; c++)
                if (z0 + c < (code[k] >> 1)) f(c, h[k][c], code[k] & 1);
    }
}

// Phase 1: a1 + a2 + a3 + b1v + b1h + b2.  Before the barrier every thread issues all of its loads
// (cluster gathers for tvert, edge gathers for b1h, its own column); after it the vertical 3-point
// stencil of tvert is read from LDS and the limiter ratios are stored.
// The block's NodeRec records (one coalesced 16-byte-per-thread sweep) into LDS after `lds_base`.
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

template <int VLIMIT, int C, int RB, int EB, bool NT>
__global__ __launch_bounds__(1024) void k_p1(MeshPlanDev mp, P1Args a, int G, float invS)
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
    const int nw = col ? max(0, min(C, Ln - z0)) : 0;  // wet cells of this thread
    real vx[C], vn[C], p[C], m[C];
#pragma unroll
    for (int c = 0; c < C; c++) vx[c] = vn[c] = p[c] = m[c] = 0.;
    size_t b = 0, ab = 0;
    if (nw > 0) {
        b = (size_t)ni.n * L + z0;
        ab = (size_t)ni.n * a.nl + z0;
        real v[C + 1];
#pragma unroll
        for (int c = 0; c <= C; c++) v[c] = (c == 0 || c < nw + 1) ? ld1_s<NT>(a.adf_v + ab + c) : 0.;
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
        cluster_bound<C, RB>(recs[j].ring, 0, min(nr, kRecRing), a.LO, a.ttf, z0, L, vx, vn);
        if (nr > kRecRing) cluster_bound<C, RB>(mp.p_ring, ni.r0 + kRecRing, ni.r1, a.LO, a.ttf, z0, L, vx, vn);
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
    stv_s<C, NT>(a.plus + b, op, nw);
    stv_s<C, NT>(a.minus + b, om, nw);
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
    const int k = group_tracer(trs.n, tr, c_tracer_major & 2) * G + j;
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

// Same, U consecutive edge groups per block: every einfo load of the U groups is issued, then every
// data load, so a thread keeps U x 5 loads in flight instead of 5 (memory-level parallelism), and
// the grid has U times fewer blocks.  NT: fct_adf_h streamed with non-temporal loads/stores so the
// gathered plus/minus columns keep the L2.
// U edge groups starting at group `ug` (relative to einfo) of one tracer.
template <int C, int U, bool NT>
__device__ __forceinline__ void b3h_groups(const int4 *__restrict__ einfo, int n_edges, int L, int G, float invS,
                                           const real *__restrict__ plus, const real *__restrict__ minus,
                                           real *__restrict__ adf_h, int ug)
{
    int j, u;
    slot_of(threadIdx.x, L / C, invS, j, u);
    if (j >= G) return;
    const int z0 = C * u;
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
            ldv_s<C, NT>(adf_h + (size_t)ei[q].w * L + z0, f[q]);
            const size_t i1 = (size_t)ei[q].x * L + z0, i2 = (size_t)ei[q].y * L + z0;
            ldv<C>(plus + i1, p1[q]);
            ldv<C>(minus + i1, m1[q]);
            ldv<C>(plus + i2, p2[q]);
            ldv<C>(minus + i2, m2[q]);
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

template <int C, int U, bool NT>
__global__ __launch_bounds__(1024) void k_b3h_u(const int4 *__restrict__ einfo, int n_edges, int L,
                                                int G, float invS, const real *__restrict__ plus,
                                                const real *__restrict__ minus,
                                                real *__restrict__ adf_h, Tracers trs)
{
    int tr;
    const int ug = group_tracer(trs.n, tr, c_tracer_major & 2);
    b3h_groups<C, U, NT>(einfo, n_edges, L, G, invS, plus + tr * trs.node, minus + tr * trs.node,
                         adf_h + tr * trs.edge, ug);
}

// Phase 2, nodes: b3v + cv + ch, G node columns per block.  fct_adf_h already holds the b3-limited
// fluxes (k_b3h_g ran first, as in docs/refactoring.md:237-314).  The limited vertical flux of the
// interface below a thread's levels is recomputed in-thread from plus/minus (the bottom interface
// nlev-1 is never limited); the barrier orders every raw fct_adf_v read of the block before its
// writes.
// The node work of phase 2 for the block's G columns (records staged): see k_p2.  COH: fct_adf_h
// read with agent-coherent loads (the persistent phase 2 publishes it inside the launch).
template <int C, int KB, bool NT, bool COH>
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
            for_edges<C, KB, COH>(recs[j].edge, 0, min(ne, kRecEdge), a.adf_h, z0, L, add);
            if (ne > kRecEdge) for_edges<C, KB, COH>(mp.p_edges, ni.e0 + kRecEdge, ni.e1, a.adf_h, z0, L, add);
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

template <int C, int KB, bool NT>
__global__ __launch_bounds__(1024) void k_p2(MeshPlanDev mp, P2Args a, int G, float invS)
{
    extern __shared__ real lds[];  // NodeRec[G]
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
    }
    const int ncol = min(G, a.count - first);
    const NodeRec *recs = stage_records(a.nodes, first, ncol, lds);
    p2_node_work<C, KB, NT, false>(mp, a, recs, ncol, invS);
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

// Edge gathers with the b3-horizontal limiter applied in-thread: for kBatch edges at a time the raw
// flux and the other endpoint's plus/minus are loaded, then f(c, limited flux, second) runs in
// ascending edge order.  (pn, mn: this node's plus/minus at the thread's levels.)
template <int C, int kBatch, class F>
__device__ __forceinline__ void for_edges_limited(const EdgeRef *__restrict__ edges, int e0, int e1,
                                                  const real *__restrict__ adf_h,
                                                  const real *__restrict__ plus,
                                                  const real *__restrict__ minus, const real (&pn)[C],
                                                  const real (&mn)[C], int z0, int L, F &&f)
{
    for (int k0 = e0; k0 < e1; k0 += kBatch) {
        EdgeRef er[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; k++) er[k] = (k0 + k < e1) ? edges[k0 + k] : EdgeRef{0, 0, 0};
        real h[kBatch][C], po[kBatch][C], mo[kBatch][C];
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            if (z0 < (er[k].code >> 1)) {
                ldv<C>(adf_h + (size_t)er[k].edge * L + z0, h[k]);
                ldv<C>(plus + (size_t)er[k].other * L + z0, po[k]);
                ldv<C>(minus + (size_t)er[k].other * L + z0, mo[k]);
            }
        }
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            const int lev = er[k].code >> 1, second = er[k].code & 1;
#pragma unroll
            for (int c = 0; c < C; c++) {
                if (z0 + c >= lev) continue;
                // docs/refactoring.md:246-257 with (n1, n2) = (other, this) when second
                const real ae = second ? b3h_factor(h[k][c], po[k][c], mo[k][c], pn[c], mn[c])
                                       : b3h_factor(h[k][c], pn[c], mn[c], po[k][c], mo[k][c]);
                f(c, ae * h[k][c], second);
            }
        }
    }
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
            auto add = [&](int c, real h, int second) {
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
            const int ne = ni.e1 - ni.e0;
            for (int k = 0; k < ne; k++) {  // ascending edge order, as the Fortran edge loop
                const EdgeRef er = k < kRecEdge ? recs[j].edge[k] : mp.p_edges[ni.e0 + k];
                const int lev = er.code >> 1, second = er.code & 1;
                if (z0 >= lev) continue;
                const int other = a.edges[2 * er.edge + (second ? 0 : 1)] - 1;
                real h[C], po[C], mo[C];
                ldv<C>(a.adf_h + (size_t)er.edge * L + z0, h);
                ldv<C>(a.plus + (size_t)other * L + z0, po);
                ldv<C>(a.minus + (size_t)other * L + z0, mo);
#pragma unroll
                for (int c = 0; c < C; c++) {
                    if (z0 + c >= lev) continue;
                    const real ae = second ? b3h_factor(h[c], po[c], mo[c], pp[c + 1], mm[c + 1])
                                           : b3h_factor(h[c], pp[c + 1], mm[c + 1], po[c], mo[c]);
                    const real lh = ae * h[c];
                    lo[c] = second ? lo[c] - lh * a.dt / ar[c] / hnn[c] : lo[c] + lh * a.dt / ar[c] / hnn[c];
                }
            }
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
    const int k = group_tracer(trs.n, tr, c_tracer_major & 2) * G + j;
    if (j >= G || k >= n_edges) return;
    plus += tr * trs.node;
    minus += tr * trs.node;
    adf_h += tr * trs.edge;
    adf_h2 += tr * trs.edge;
    const int4 ei = einfo[k];
    const size_t i = (size_t)ei.w * L + z0;
    const size_t i1 = (size_t)ei.x * L + z0, i2 = (size_t)ei.y * L + z0;
    real f[C], h2[C], p1[C], m1[C], p2[C], m2[C];
    ldv<C>(adf_h + i, f);
    ldv<C>(adf_h2 + i, h2);
    if (z0 < ei.z) {
        ldv<C>(plus + i1, p1);
        ldv<C>(minus + i1, m1);
        ldv<C>(plus + i2, p2);
        ldv<C>(minus + i2, m2);
    }
#pragma unroll
    for (int c = 0; c < C; c++)
        if (z0 + c < ei.z) h2[c] = (1.0 - b3h_factor(f[c], p1[c], m1[c], p2[c], m2[c])) * f[c];
    stv<C>(adf_h2 + i, h2, C);
    stv<C>(adf_h + i, h2, C);
}

// columns per block for S slots per column: G*S fills whole waves where possible (<= 1024 threads)
int group_columns(int S)
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
    // FESOM2_GROUP_SHIFT = k: 2^k times as many columns per block (k < 0: fewer; A/B measurements,
    // results do not depend on it)
    static const int shift = [] {
        const char *e = getenv("FESOM2_GROUP_SHIFT");
        return e ? atoi(e) : 0;
    }();
    for (int k = 0; k < shift && best * 2 * S <= 1024; k++) best *= 2;
    for (int k = 0; k > shift && best > 1; k--) best /= 2;
    return best;
}

static inline unsigned threads_for(int G, int S) { return (unsigned)(((G * S + kWave - 1) / kWave) * kWave); }

// levels per thread: 2 when columns are 16-byte aligned (L even), else 1
static inline int levels_per_thread(int L)
{
    const char *e = getenv("FESOM2_CPT");
    if (e && atoi(e) == 1) return 1;
    return (L % 2 == 0) ? 2 : 1;
}

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
#define F2A_LAUNCH_GROUPS(kernel, groups, G, L, lds_bytes, s, ...)                                       \
    do {                                                                                                \
        init_swizzle();                                                                                 \
        if ((groups) > 0)                                                                               \
            hipLaunchKernelGGL(kernel, dim3((unsigned)(groups)), dim3(threads_for(G, L)), (lds_bytes), \
                               (s), __VA_ARGS__);                                                       \
        return hipGetLastError();                                                                       \
    } while (0)

static int env_int(const char *name, int dflt)
{
    const char *e = getenv(name);
    return e ? atoi(e) : dflt;
}

template <int C, int RB, int EB>
static hipError_t p1_launch(const MeshPlanDev &mp, const P1Args &a, hipStream_t s, int G, int S, long groups)
{
    const float invS = 1.0f / (float)S;
    const size_t lds = 2 * (size_t)G * (a.nl - 1) * sizeof(real) + (size_t)G * sizeof(NodeRec);
    const bool NT = (env_int("FESOM2_NT", 2) & 1) != 0;
    if (a.vlimit == 2) F2A_LAUNCH_GROUPS((k_p1<2, C, RB, EB, false>), groups, G, S, lds, s, mp, a, G, invS);
    if (a.vlimit == 3) F2A_LAUNCH_GROUPS((k_p1<3, C, RB, EB, false>), groups, G, S, lds, s, mp, a, G, invS);
    if (NT) F2A_LAUNCH_GROUPS((k_p1<1, C, RB, EB, true>), groups, G, S, lds, s, mp, a, G, invS);
    F2A_LAUNCH_GROUPS((k_p1<1, C, RB, EB, false>), groups, G, S, lds, s, mp, a, G, invS);
}

int fused_group_columns(int nl)
{
    const int L = nl - 1;
    return group_columns(L / levels_per_thread(L));
}

hipError_t launch_p1_fused(const MeshPlanDev &mp, const P1Args &a, hipStream_t s)
{
    const int L = a.nl - 1, C = levels_per_thread(L), S = L / C, G = group_columns(S);
    const long groups = (long)(a.n_owned + G - 1) / G * a.tr.n;
    // cluster along the edge list (FESOM2_P1_EDGE=1 where the plan verified it; measured equal at
    // EB = 1, slower at EB >= 2: DESIGN.md §3)
    if (mp.edge_cluster && env_int("FESOM2_P1_EDGE", 0)) {
        const size_t lds = 2 * (size_t)G * L * sizeof(real) + (size_t)G * sizeof(NodeRec);
        const float invS = 1.0f / (float)S;
        const int EB = env_int("FESOM2_P1E_EB", 2);
#define F2A_P1E(CC, EBV)                                                                                        \
        if (a.vlimit == 2) F2A_LAUNCH_GROUPS((k_p1e<2, CC, EBV>), groups, G, S, lds, s, mp, a, G, invS);  \
        if (a.vlimit == 3) F2A_LAUNCH_GROUPS((k_p1e<3, CC, EBV>), groups, G, S, lds, s, mp, a, G, invS);  \
        F2A_LAUNCH_GROUPS((k_p1e<1, CC, EBV>), groups, G, S, lds, s, mp, a, G, invS);
        if (C == 2) {
            if (EB == 1) { F2A_P1E(2, 1) }
            if (EB == 4) { F2A_P1E(2, 4) }
            F2A_P1E(2, 2)
        }
        F2A_P1E(1, 2)
#undef F2A_P1E
    }
    // staged cluster (FESOM2_P1_STAGE=1; vlimit 1 only; measured slower at G = 8)
    if (a.vlimit == 1 && mp.stage_max > 0 && mp.stage_G == G && env_int("FESOM2_P1_STAGE", 0)) {
        const int U = std::max(mp.stage_max, G);
        const size_t lds = 2 * (size_t)U * L * sizeof(real) + (size_t)G * sizeof(NodeRec);
        const float invS = 1.0f / (float)S;
        const int EB = env_int("FESOM2_P1S_EB", 2);
        const int KS = (mp.stage_max * S + (int)threads_for(G, S) - 1) / (int)threads_for(G, S);  // items per thread
        if (C == 2 && KS <= 8) {
#define F2A_P1S(EBV, KSV) \
            if (EB == EBV && KS <= KSV) F2A_LAUNCH_GROUPS((k_p1s<2, EBV, KSV>), groups, G, S, lds, s, mp, a, G, invS, U);
            F2A_P1S(2, 2) F2A_P1S(2, 4) F2A_P1S(2, 6) F2A_P1S(2, 8)
            F2A_P1S(4, 2) F2A_P1S(4, 4) F2A_P1S(4, 6) F2A_P1S(4, 8)
#undef F2A_P1S
        }
    }
    // batch sizes of the cluster / edge gathers (FESOM2_P1_BATCH = 10*RB + EB; measured)
    switch (env_int("FESOM2_P1_BATCH", 22)) {
    case 44: return C == 2 ? p1_launch<2, 4, 4>(mp, a, s, G, S, groups) : p1_launch<1, 4, 4>(mp, a, s, G, S, groups);
    case 24: return C == 2 ? p1_launch<2, 2, 4>(mp, a, s, G, S, groups) : p1_launch<1, 2, 4>(mp, a, s, G, S, groups);
    case 42: return C == 2 ? p1_launch<2, 4, 2>(mp, a, s, G, S, groups) : p1_launch<1, 4, 2>(mp, a, s, G, S, groups);
    case 88: return C == 2 ? p1_launch<2, 8, 8>(mp, a, s, G, S, groups) : p1_launch<1, 8, 8>(mp, a, s, G, S, groups);
    default: return C == 2 ? p1_launch<2, 2, 2>(mp, a, s, G, S, groups) : p1_launch<1, 2, 2>(mp, a, s, G, S, groups);
    }
}

hipError_t launch_p2_fused(const MeshPlanDev &mp, const P2Args &a, hipStream_t s)
{
    const int L = a.nl - 1;
    // levels per thread of the node kernel: FESOM2_P2_CPT (1 or 2; default as the other kernels)
    const int C = (L % 2 == 0 && env_int("FESOM2_P2_CPT", levels_per_thread(L)) == 2) ? 2 : 1;
    const int S = L / C, G = group_columns(S);
    const long groups = (long)(a.count + G - 1) / G * a.tr.n;
    const float invS = 1.0f / (float)S;
    const int KB = env_int("FESOM2_P2_BATCH", 4);
    const size_t lds = (size_t)G * sizeof(NodeRec);
    if (C == 2) {
        const bool NT = (env_int("FESOM2_NT", 2) & 2) != 0;  // measured: p2 streams non-temporal (-2 %)
        if (NT) F2A_LAUNCH_GROUPS((k_p2<2, 4, true>), groups, G, S, lds, s, mp, a, G, invS);
        if (KB == 8) F2A_LAUNCH_GROUPS((k_p2<2, 8, false>), groups, G, S, lds, s, mp, a, G, invS);
        F2A_LAUNCH_GROUPS((k_p2<2, 4, false>), groups, G, S, lds, s, mp, a, G, invS);
    }
    if ((env_int("FESOM2_NT", 2) & 2) != 0) F2A_LAUNCH_GROUPS((k_p2<1, 4, true>), groups, G, S, lds, s, mp, a, G, invS);
    if (KB == 8) F2A_LAUNCH_GROUPS((k_p2<1, 8, false>), groups, G, S, lds, s, mp, a, G, invS);
    if (KB == 2) F2A_LAUNCH_GROUPS((k_p2<1, 2, false>), groups, G, S, lds, s, mp, a, G, invS);
    F2A_LAUNCH_GROUPS((k_p2<1, 4, false>), groups, G, S, lds, s, mp, a, G, invS);
}

hipError_t launch_b3h_fused(const MeshPlanDev &mp, int nl, int begin, int count, const real *plus,
                            const real *minus, real *adf_h, const Tracers &tr, hipStream_t s)
{
    return launch_b3h_edges(mp.p_edge_info + begin, count, nl, plus, minus, adf_h, tr, s);
}

hipError_t launch_b3h_edges(const int4 *ei, int count, int nl, const real *plus, const real *minus,
                            real *adf_h, const Tracers &tr, hipStream_t s)
{
    const int L = nl - 1;
    int C = levels_per_thread(L);
    if (C == 2 && L % 4 == 0 && env_int("FESOM2_B3H_CPT", 2) == 4) C = 4;  // 4 levels: 2 x 16 B per array
    const int S = L / C, G = group_columns(S);
    const long groups = (count + G - 1) / G;
    const float invS = 1.0f / (float)S;
    const long tg = groups * tr.n;
    if (C == 4) F2A_LAUNCH_GROUPS(k_b3h_g<4>, tg, G, S, 0, s, ei, count, L, G, invS, plus, minus, adf_h, tr);
    if (C == 2) {
        // U edge groups per block, fct_adf_h non-temporal (FESOM2_B3H_U / FESOM2_B3H_NT; measured)
        const int U = env_int("FESOM2_B3H_U", 2);
        const bool NT = env_int("FESOM2_B3H_NT", 1) != 0;
        const long ug = (groups + U - 1) / U * tr.n;
#define F2A_B3H_U(UU)                                                                                   \
        if (U == UU) {                                                                                  \
            if (NT) F2A_LAUNCH_GROUPS((k_b3h_u<2, UU, true>), ug, G, S, 0, s, ei, count, L, G, invS, plus, minus, adf_h, tr); \
            F2A_LAUNCH_GROUPS((k_b3h_u<2, UU, false>), ug, G, S, 0, s, ei, count, L, G, invS, plus, minus, adf_h, tr); \
        }
        F2A_B3H_U(2)
        F2A_B3H_U(4)
        F2A_B3H_U(8)
#undef F2A_B3H_U
        if (NT) F2A_LAUNCH_GROUPS((k_b3h_u<2, 1, true>), tg, G, S, 0, s, ei, count, L, G, invS, plus, minus, adf_h, tr);
        F2A_LAUNCH_GROUPS(k_b3h_g<2>, tg, G, S, 0, s, ei, count, L, G, invS, plus, minus, adf_h, tr);
    }
    {
        // one level per thread (odd L): the same two-groups-per-block, non-temporal form
        const int U = env_int("FESOM2_B3H_U", 2);
        const bool NT = env_int("FESOM2_B3H_NT", 1) != 0;
        const long ug = (groups + U - 1) / U * tr.n;
        if (U == 2 && NT) F2A_LAUNCH_GROUPS((k_b3h_u<1, 2, true>), ug, G, S, 0, s, ei, count, L, G, invS, plus, minus, adf_h, tr);
        if (U == 4 && NT) F2A_LAUNCH_GROUPS((k_b3h_u<1, 4, true>), ug, G, S, 0, s, ei, count, L, G, invS, plus, minus, adf_h, tr);
    }
    F2A_LAUNCH_GROUPS(k_b3h_g<1>, tg, G, S, 0, s, ei, count, L, G, invS, plus, minus, adf_h, tr);
}

hipError_t launch_p2_fused_b3h(const MeshPlanDev &mp, const P2Args &a, hipStream_t s)
{
    const int L = a.nl - 1, C = levels_per_thread(L), S = L / C, G = group_columns(S);
    const long groups = (long)(a.count + G - 1) / G * a.tr.n;
    const float invS = 1.0f / (float)S;
    const size_t lds = (size_t)G * (sizeof(NodeRec) + sizeof(unsigned));
    const int KB = env_int("FESOM2_P2F_BATCH", 2);
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
    if (getenv("FESOM2_PLAN_STATS")) fprintf(stderr, "fesom2-accelerate: wavefront grid %ld (%d per CU)\n", grid, per_cu);
    grid = std::max<long>(kWfStreams, grid / kWfStreams * kWfStreams);
    init_swizzle();
    if (C == 2)
        hipLaunchKernelGGL((k_p2w<2, 4>), dim3((unsigned)grid), dim3(threads), lds, s, mp, a, state, G, invS);
    else
        hipLaunchKernelGGL((k_p2w<1, 4>), dim3((unsigned)grid), dim3(threads), lds, s, mp, a, state, G, invS);
    return hipGetLastError();
}

hipError_t launch_p2_iter(const MeshPlanDev &mp, const P2IterArgs &a, hipStream_t s)
{
    const int L = a.nl - 1, C = levels_per_thread(L), S = L / C, G = group_columns(S);
    const long groups = (long)(a.count + G - 1) / G * a.tr.n;
    const float invS = 1.0f / (float)S;
    const size_t lds = (size_t)G * sizeof(NodeRec);
    if (C == 2) F2A_LAUNCH_GROUPS((k_p2_iter<2>), groups, G, S, lds, s, mp, a, G, invS);
    F2A_LAUNCH_GROUPS((k_p2_iter<1>), groups, G, S, lds, s, mp, a, G, invS);
}

hipError_t launch_b3h_iter(const MeshPlanDev &mp, int nl, const real *plus, const real *minus, real *adf_h,
                           real *adf_h2, const Tracers &tr, hipStream_t s)
{
    const int L = nl - 1, C = levels_per_thread(L), S = L / C, G = group_columns(S);
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
