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
// Mapping: one wave64 per node column (or element / edge), lanes over vertical levels, 4 waves per
// 256-thread workgroup, and an XCD-aware block swizzle so each XCD's L2 walks a contiguous range
// of the (spatially sorted) mesh: neighbouring columns gathered by the cluster/edge loops are then
// L2/Infinity-Cache hits rather than HBM re-reads.
#include "f2a_internal.hpp"
#include <cmath>

namespace f2a {

#define RMAX(a, b) (((a) < (b)) ? (b) : (a))  // std::max(a, b)
#define RMIN(a, b) (((b) < (a)) ? (b) : (a))  // std::min(a, b)

static constexpr int kWave = 64;
static constexpr int kWavesPerBlock = 4;
static constexpr int kBlock = kWave * kWavesPerBlock;

// Bijective XCD-aware swizzle: blocks b and b+8 share an XCD (round-robin dispatch), so hand each
// residue class a contiguous range of tiles.  Speed only, never correctness.
__device__ __forceinline__ int xcd_tile(int b, int G)
{
    const int q = G >> 3, r = G & 7, x = b & 7, k = b >> 3;
    return x * q + (x < r ? x : r) + k;
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
    for (int k = e0; k < e1; k++) lmax = max(lmax, mp.edges[k].lev);
    const size_t b = (size_t)n * L;
    for (int z = lane; z < lmax; z += kWave) {
        real p = plus[b + z], m = minus[b + z];
        for (int k = e0; k < e1; k++) {
            const EdgeRef er = mp.edges[k];
            if (z < er.lev) {
                const real h = adf_h[(size_t)er.edge * L + z];
                if (er.flags & 1) {
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
    for (int k = e0; k < e1; k++) lmax = max(lmax, mp.edges[k].lev);
    const size_t b = (size_t)n * L, a = (size_t)n * (L + 1);
    for (int z = lane; z < lmax; z += kWave) {
        const real dta = dt / area[a + z];
        real d = del_h[b + z];
        for (int k = e0; k < e1; k++) {
            const EdgeRef er = mp.edges[k];
            if (z < er.lev) {
                const real h = adf_h[(size_t)er.edge * L + z];
                d = (er.flags & 1) ? d - h * dta : d + h * dta;
            }
        }
        del_h[b + z] = d;
    }
}

// ============================================================================ fused kernels

// Phase 1: a1 + a2 + a3 + b1v + b1h + b2 for one owned node per wave.
// The cluster bound tvert(z) = max over adjacent elements e of UV_rhs(e, z) is computed straight
// from ttf/LO over the node's cluster (RingRef list): a cluster node k contributes on levels
// z < ring.lev (the element-level mask of a2), and the a2 fill -bignumber enters wherever some
// adjacent element is dry (z >= zdry).  max/min are exact, so regrouping them leaves the values of
// reference.cpp:321-378 unchanged.  The vertical 3-point stencil reads tvert from LDS.
template <int VLIMIT>
__global__ __launch_bounds__(kBlock) void k_p1(MeshPlanDev mp, P1Args a)
{
    extern __shared__ real lds[];
    const int n = wave_item();
    if (n >= a.n_owned) return;
    const int lane = threadIdx.x & 63;
    const int L = a.nl - 1;
    real *tvx = lds + (threadIdx.x >> 6) * 2 * L;
    real *tvn = tvx + L;
    const int Ln = a.nlev_nod[n] - 1;
    const int r0 = mp.ring_ptr[n], r1 = mp.ring_ptr[n + 1];
    const int zd = mp.zdry[n];
    for (int z = lane; z < Ln; z += kWave) {
        real vx = (z >= zd) ? -a.big : -INFINITY;
        real vn = (z >= zd) ? a.big : INFINITY;
        for (int r = r0; r < r1; r++) {
            const RingRef rr = mp.ring[r];
            if (z < rr.lev) {
                const size_t i = (size_t)rr.node * L + z;
                const real lo = a.LO[i], t = a.ttf[i];
                vx = RMAX(vx, RMAX(lo, t));
                vn = RMIN(vn, RMIN(lo, t));
            }
        }
        tvx[z] = vx;
        tvn[z] = vn;
    }
    wave_lds_sync();
    const int e0 = mp.edge_ptr[n], e1 = mp.edge_ptr[n + 1];
    const size_t b = (size_t)n * L, ab = (size_t)n * a.nl;
    for (int z = lane; z < Ln; z += kWave) {
        const real lo = a.LO[b + z];
        real tm, tn;
        if (VLIMIT == 1) {
            if (z == 0 || z == Ln - 1) {
                tm = tvx[z];
                tn = tvn[z];
            } else {
                tm = RMAX(RMAX(tvx[z - 1], tvx[z]), tvx[z + 1]);
                tn = RMIN(RMIN(tvn[z - 1], tvn[z]), tvn[z + 1]);
            }
        } else {
            tm = tvx[z];
            tn = tvn[z];
            if (z >= 1 && z < Ln - 1) {
                const real c0 = RMAX(a.LO[b + z - 1], a.ttf[b + z - 1]);
                const real c1 = RMAX(lo, a.ttf[b + z]);
                const real c2 = RMAX(a.LO[b + z + 1], a.ttf[b + z + 1]);
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
        const real fmx = tm - lo, fmn = tn - lo;
        const real v0 = a.adf_v[ab + z], v1 = a.adf_v[ab + z + 1];
        real p = RMAX(0., v0) + RMAX(0., -v1);
        real m = RMIN(0., v0) + RMIN(0., -v1);
        for (int k = e0; k < e1; k++) {
            const EdgeRef er = mp.edges[k];
            if (z < er.lev) {
                const real h = a.adf_h[(size_t)er.edge * L + z];
                if (er.flags & 1) {
                    p += RMAX(0., -h);
                    m += RMIN(0., -h);
                } else {
                    p += RMAX(0., h);
                    m += RMIN(0., h);
                }
            }
        }
        const real ai = a.area_inv[ab + z];
        real flux = p * a.dt * ai + a.eps;
        a.plus[b + z] = RMIN(1., fmx / flux);
        flux = m * a.dt * ai - a.eps;
        a.minus[b + z] = RMIN(1., fmn / flux);
    }
}

// Phase 2 node part: b3v + cv + ch for one owned node per wave.  fct_adf_h must already hold the
// b3-limited fluxes (k_b3h runs first, as in docs/refactoring.md:237-314).  The limited vertical
// flux of interface z+1 is recomputed in-lane from plus/minus(z, z+1) (bottom interface nlev-1 is
// never limited), so the column is read once and written once.
__global__ __launch_bounds__(kBlock) void k_p2(MeshPlanDev mp, P2Args a)
{
    int i = wave_item();
    if (i >= a.count) return;
    const int n = a.nodes ? __builtin_amdgcn_readfirstlane(a.nodes[i]) : i;
    const int lane = threadIdx.x & 63;
    const int L = a.nl - 1;
    const int Ln = a.nlev_nod[n] - 1;
    const size_t b = (size_t)n * L, ab = (size_t)n * a.nl;
    const int e0 = mp.edge_ptr[n], e1 = mp.edge_ptr[n + 1];
    const int top = Ln > 1 ? Ln : 1;
    for (int z = lane; z < top; z += kWave) {
        const real pz = a.plus[b + z], mz = a.minus[b + z];
        const real pm = z ? a.plus[b + z - 1] : 0., mm = z ? a.minus[b + z - 1] : 0.;
        const real f0 = a.adf_v[ab + z], f1 = a.adf_v[ab + z + 1];
        const real l0 = b3v_factor(z, f0, pm, mm, pz, mz) * f0;
        real l1 = f1;
        if (z + 1 < Ln) l1 = b3v_factor(z + 1, f1, pz, mz, a.plus[b + z + 1], a.minus[b + z + 1]) * f1;
        a.adf_v[ab + z] = l0;
        if (z >= Ln) continue;  // Ln == 0: only the Fortran's nz = 1 limiting applies
        const real ar = a.area[ab + z];
        const real dta = a.dt / ar;
        real t = a.del_v[b + z] - a.ttf[b + z] * a.hnode[b + z];
        t = t + a.LO[b + z] * a.hnode_new[b + z];
        t = t + (l0 - l1) * dta;
        a.del_v[b + z] = t;
        real d = a.del_h[b + z];
        for (int k = e0; k < e1; k++) {
            const EdgeRef er = mp.edges[k];
            if (z < er.lev) {
                const real h = a.adf_h[(size_t)er.edge * L + z];
                d = (er.flags & 1) ? d - h * dta : d + h * dta;
            }
        }
        a.del_h[b + z] = d;
    }
    // levels the node's edges carry beyond its own column never occur on a consistent mesh
    // (nlevels_nod2D = max over adjacent elements), so no second loop is needed.
}

// ============================================================================ halo pack / unpack

__global__ __launch_bounds__(kBlock) void k_pack(const int *__restrict__ nodes, int count, int L,
                                                 const real *__restrict__ plus,
                                                 const real *__restrict__ minus,
                                                 real *__restrict__ buf)
{
    const int i = wave_item();
    if (i >= count) return;
    const size_t src = (size_t)nodes[i] * L, dst = (size_t)i * 2 * L;
    for (int z = threadIdx.x & 63; z < L; z += kWave) {
        buf[dst + z] = plus[src + z];
        buf[dst + L + z] = minus[src + z];
    }
}

__global__ __launch_bounds__(kBlock) void k_unpack(const int *__restrict__ nodes, int count, int L,
                                                   const real *__restrict__ buf,
                                                   real *__restrict__ plus,
                                                   real *__restrict__ minus)
{
    const int i = wave_item();
    if (i >= count) return;
    const size_t dst = (size_t)nodes[i] * L, src = (size_t)i * 2 * L;
    for (int z = threadIdx.x & 63; z < L; z += kWave) {
        plus[dst + z] = buf[src + z];
        minus[dst + z] = buf[src + L + z];
    }
}

// ============================================================================ launchers

#define F2A_LAUNCH(kernel, items, lds_bytes, s, ...)                                    \
    do {                                                                                \
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

hipError_t launch_p1_fused(const MeshPlanDev &mp, const P1Args &a, hipStream_t s)
{
    const size_t lds = (size_t)kWavesPerBlock * 2 * (a.nl - 1) * sizeof(real);
    if (a.vlimit == 2) F2A_LAUNCH(k_p1<2>, a.n_owned, lds, s, mp, a);
    if (a.vlimit == 3) F2A_LAUNCH(k_p1<3>, a.n_owned, lds, s, mp, a);
    F2A_LAUNCH(k_p1<1>, a.n_owned, lds, s, mp, a);
}

hipError_t launch_p2_fused(const MeshPlanDev &mp, const P2Args &a, hipStream_t s)
{
    F2A_LAUNCH(k_p2, a.count, 0, s, mp, a);
}

hipError_t launch_halo_pack(const int *nodes, int count, int L, const real *plus,
                            const real *minus, real *buf, hipStream_t s)
{
    F2A_LAUNCH(k_pack, count, 0, s, nodes, count, L, plus, minus, buf);
}

hipError_t launch_halo_unpack(const int *nodes, int count, int L, const real *buf, real *plus,
                              real *minus, hipStream_t s)
{
    F2A_LAUNCH(k_unpack, count, 0, s, nodes, count, L, buf, plus, minus);
}

}  // namespace f2a
