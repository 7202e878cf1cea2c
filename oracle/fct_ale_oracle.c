/*
 * fct_ale_oracle.c -- CPU restatement of the FCT-ALE limiter (TEST INFRASTRUCTURE ONLY).
 *
 * This file is the parity oracle for the HIP engine in fesom2-accelerate_amd/.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product path never
 * links or calls it.
 *
 * What it restates (reference = ESiWACE-S1/fesom2-accelerate, read-only at /root/reference):
 *   a1  fct_ale_a1_reference_   src/reference.cpp:306-319
 *   a2  fct_ale_a2_reference_   src/reference.cpp:321-351
 *   a3  fct_ale_a3_reference_   src/reference.cpp:353-401   (includes b1-vertical, :393-399)
 *   a4  fct_ale_a4_reference_   src/reference.cpp:403-438   (b1-horizontal :406-425, b2 :426-437)
 *   pre_comm sequencer          src/reference.cpp:289-304   (28-argument header form, .h:235)
 *   b3v  docs/refactoring.md:204-233   = kernels/fct_ale_b3_vertical.cu:2-46, numpy fct_ale_b3_vertical.py:163-181
 *   b3h  docs/refactoring.md:237-263   = kernels/fct_ale_b3_horizontal.cu:2-42, numpy fct_ale_b3_horizontal.py:76-101
 *   cv   docs/refactoring.md:295-300   in the expression order of kernels/fct_ale_c_vertical.cu:9-12
 *        (= numpy fct_ale_c_vertical.py:44): ((del - ttf*hnode) + LO*hnode_new) + (adf_v[z]-adf_v[z+1])*(dt/area)
 *   ch   docs/refactoring.md:302-314   in the expression order of kernels/fct_ale_c_horizontal.cu:22-26
 *        (= numpy fct_ale_c_horizontal.py:69-70): del[n1] += adf_h*(dt/area[n1]); del[n2] -= adf_h*(dt/area[n2])
 *   vlimit 2/3 a3 variants      docs/refactoring.md:113-148 (Fortran; not in reference.cpp, which stops after a2)
 *   iter_yn branch              docs/refactoring.md:227-229, :258-260, :265-290
 *
 * Parity pin: a1..a4 are checked bit-for-bit against reference.cpp compiled from
 * /root/reference/src/reference.cpp (oracle/Makefile -> oracle/_ref/) and against the committed
 * fixtures in tests/golden/ (made by tests/golden/make_golden.py).  b3/c are pinned against the
 * reference's numpy reference() functions through the same fixtures.
 *
 * Layout (Fortran column-major, 0-based here): node arrays (L, nodes) item = n*L + z with L = nl-1;
 * fct_adf_v / area / area_inv (nl, nodes) item = n*nl + z; fct_adf_h (L, edges) item = e*L + z;
 * UV_rhs (2, L, elem) item = 2*(e*L + z) + {0 max, 1 min}.  Connectivity is 1-based (Fortran).
 *
 * max/min follow std::max / std::min exactly (first argument wins ties), see RMAX/RMIN.
 * Build with -ffp-contract=off so no multiply-add is fused (the x86-64 reference build has none).
 */
#include <stdlib.h>
#include <string.h>

#define RMAX(a, b) (((a) < (b)) ? (b) : (a)) /* std::max(a, b) */
#define RMIN(a, b) (((b) < (a)) ? (b) : (a)) /* std::min(a, b) */

/* a1: reference.cpp:306-319 (Fortran docs/refactoring.md:47-52) */
void oracle_a1(int nNodes, const int *nlev_nod, int nl, double *ttf_max, double *ttf_min,
               const double *LO, const double *ttf)
{
    const int L = nl - 1;
    for (int n = 0; n < nNodes; n++)
        for (int z = 0; z < nlev_nod[n] - 1; z++) {
            long i = (long)n * L + z;
            ttf_max[i] = RMAX(LO[i], ttf[i]);
            ttf_min[i] = RMIN(LO[i], ttf[i]);
        }
}

/* a2: reference.cpp:321-351 (Fortran :58-70); fill (-big, +big) for nlev_e-1 <= z < L */
void oracle_a2(int nElem, const int *nlev_elem, int nl, double *UV_rhs, const int *elem2D_nodes,
               const double *ttf_max, const double *ttf_min, double big)
{
    const int L = nl - 1;
    for (int e = 0; e < nElem; e++) {
        const long k0 = (long)(elem2D_nodes[3 * e] - 1) * L;
        const long k1 = (long)(elem2D_nodes[3 * e + 1] - 1) * L;
        const long k2 = (long)(elem2D_nodes[3 * e + 2] - 1) * L;
        for (int z = 0; z < nlev_elem[e] - 1; z++) {
            long u = 2 * ((long)e * L + z);
            UV_rhs[u] = RMAX(RMAX(ttf_max[k0 + z], ttf_max[k1 + z]), ttf_max[k2 + z]);
            UV_rhs[u + 1] = RMIN(RMIN(ttf_min[k0 + z], ttf_min[k1 + z]), ttf_min[k2 + z]);
        }
        if (nlev_elem[e] <= L)
            for (int z = nlev_elem[e] - 1; z < L; z++) {
                long u = 2 * ((long)e * L + z);
                UV_rhs[u] = -big;
                UV_rhs[u + 1] = big;
            }
    }
}

/* cluster bounds of a3/vlimit 1-3: tvert over nod_in_elem2D(1:num, n), reference.cpp:358-378 */
static void tvert_bounds(int n, int L, int nLevs, const double *UV_rhs, const int *nie,
                         const int *nie_num, int dim, double *tmax, double *tmin)
{
    const int nelems = nie_num[n];
    long e0 = nie[(long)n * dim] - 1;
    for (int z = 0; z < nLevs - 1; z++) {
        long u = 2 * (e0 * L + z);
        tmax[z] = UV_rhs[u];
        tmin[z] = UV_rhs[u + 1];
    }
    for (int k = 1; k < nelems; k++) {
        long ek = nie[(long)n * dim + k] - 1;
        for (int z = 0; z < nLevs - 1; z++) {
            long u = 2 * (ek * L + z);
            tmax[z] = RMAX(tmax[z], UV_rhs[u]);
            tmin[z] = RMIN(tmin[z], UV_rhs[u + 1]);
        }
    }
}

/* b1-vertical: reference.cpp:393-399 (Fortran :156-169), adf_v stride nl */
static void b1_vertical_node(int n, int L, int nLevs, double *plus, double *minus, const double *adf_v)
{
    for (int z = 0; z < nLevs - 1; z++) {
        long i = (long)n * L + z;
        long a = (long)n * (L + 1) + z;
        plus[i] = RMAX(0., adf_v[a]) + RMAX(0., -adf_v[a + 1]);
        minus[i] = RMIN(0., adf_v[a]) + RMIN(0., -adf_v[a + 1]);
    }
}

/* a3 (vlimit == 1) + b1-vertical: reference.cpp:353-401 (Fortran :77-108) */
void oracle_a3(int nNodes, const int *nlev_nod, int nl, double *ttf_max, double *ttf_min,
               const double *LO, const double *UV_rhs, double *plus, double *minus,
               const double *adf_v, const int *nie, const int *nie_num, int dim)
{
    const int L = nl - 1;
    double *tmax = (double *)calloc(L > 0 ? L : 1, sizeof(double));
    double *tmin = (double *)calloc(L > 0 ? L : 1, sizeof(double));
    for (int n = 0; n < nNodes; n++) {
        const int nLevs = nlev_nod[n];
        const long base = (long)n * L;
        tvert_bounds(n, L, nLevs, UV_rhs, nie, nie_num, dim, tmax, tmin);
        ttf_max[base] = tmax[0] - LO[base];
        ttf_min[base] = tmin[0] - LO[base];
        for (int z = 1; z < nLevs - 2; z++) {
            long i = base + z;
            ttf_max[i] = RMAX(RMAX(tmax[z - 1], tmax[z]), tmax[z + 1]) - LO[i];
            ttf_min[i] = RMIN(RMIN(tmin[z - 1], tmin[z]), tmin[z + 1]) - LO[i];
        }
        long i = base + nLevs - 2;
        ttf_max[i] = tmax[nLevs - 2] - LO[i];
        ttf_min[i] = tmin[nLevs - 2] - LO[i];
        b1_vertical_node(n, L, nLevs, plus, minus, adf_v);
    }
    free(tmax);
    free(tmin);
}

/*
 * a3 for vlimit 2 / 3 (Fortran docs/refactoring.md:113-148) + b1-vertical.  reference.cpp has no
 * vlimit 2/3 (it stops after a2 with alg_state 2, :297-303).  The Fortran's
 * `minval(fct_ttf_max(nz-1:nz+1,n))` for tvert_min (:121, :141) is restated as written.
 * fct_ttf_max/min read here are the a1 results (a3 overwrites them only in its last loop).
 */
void oracle_a3_vlimit23(int vlimit, int nNodes, const int *nlev_nod, int nl, double *ttf_max,
                        double *ttf_min, const double *LO, const double *UV_rhs, double *plus,
                        double *minus, const double *adf_v, const int *nie, const int *nie_num,
                        int dim)
{
    const int L = nl - 1;
    double *tmax = (double *)calloc(L > 0 ? L : 1, sizeof(double));
    double *tmin = (double *)calloc(L > 0 ? L : 1, sizeof(double));
    for (int n = 0; n < nNodes; n++) {
        const int nLevs = nlev_nod[n];
        const long base = (long)n * L;
        tvert_bounds(n, L, nLevs, UV_rhs, nie, nie_num, dim, tmax, tmin);
        for (int z = 1; z < nLevs - 2; z++) {
            long i = base + z;
            double vmax = RMAX(RMAX(ttf_max[i - 1], ttf_max[i]), ttf_max[i + 1]);
            double vmin = RMIN(RMIN(ttf_max[i - 1], ttf_max[i]), ttf_max[i + 1]);
            if (vlimit == 2) {
                tmax[z] = RMAX(tmax[z], vmax);
                tmin[z] = RMIN(tmin[z], vmin);
            } else {
                tmax[z] = RMIN(tmax[z], vmax);
                tmin[z] = RMAX(tmin[z], vmin);
            }
        }
        for (int z = 0; z < nLevs - 1; z++) {
            long i = base + z;
            ttf_max[i] = tmax[z] - LO[i];
            ttf_min[i] = tmin[z] - LO[i];
        }
        b1_vertical_node(n, L, nLevs, plus, minus, adf_v);
    }
    free(tmax);
    free(tmin);
}

/* b1-horizontal over all local edges: reference.cpp:406-425 (Fortran :171-186) */
void oracle_b1h(const int *nlev_elem, int nl, int nEdges, double *plus, double *minus,
                const double *adf_h, const int *edges, const int *edge_tri)
{
    const int L = nl - 1;
    for (int e = 0; e < nEdges; e++) {
        long n1 = (long)(edges[2 * e] - 1) * L;
        long n2 = (long)(edges[2 * e + 1] - 1) * L;
        int el1 = edge_tri[2 * e] - 1;
        int el2 = edge_tri[2 * e + 1] - 1;
        int nl1 = nlev_elem[el1] - 1;
        int nl2 = (el2 >= 0) ? (nlev_elem[el2] - 1) : 0;
        int maxLev = RMAX(nl1, nl2);
        for (int z = 0; z < maxLev; z++) {
            double a = adf_h[(long)e * L + z];
            plus[n1 + z] += RMAX(0., a);
            minus[n1 + z] += RMIN(0., a);
            plus[n2 + z] += RMAX(0., -a);
            minus[n2 + z] += RMIN(0., -a);
        }
    }
}

/* b2 over owned nodes: reference.cpp:426-437 (Fortran :189-197; area_inv as in reference.cpp) */
void oracle_b2(int nNodes, const int *nlev_nod, int nl, double *plus, double *minus,
               const double *area_inv, const double *ttf_max, const double *ttf_min,
               double flux_eps, double dt)
{
    const int L = nl - 1;
    for (int n = 0; n < nNodes; n++)
        for (int z = 0; z < nlev_nod[n] - 1; z++) {
            long i = (long)n * L + z;
            long ai = (long)n * (L + 1) + z;
            double flux = plus[i] * dt * area_inv[ai] + flux_eps;
            plus[i] = RMIN(1., ttf_max[i] / flux);
            flux = minus[i] * dt * area_inv[ai] - flux_eps;
            minus[i] = RMIN(1., ttf_min[i] / flux);
        }
}

/* a4 = b1-horizontal over edges + b2 over owned nodes: reference.cpp:403-438 */
void oracle_a4(int nNodes, const int *nlev_nod, const int *nlev_elem, int nl, int nEdges,
               double *plus, double *minus, const double *adf_h, const double *area_inv,
               const double *ttf_max, const double *ttf_min, const int *edges, const int *edge_tri,
               double flux_eps, double dt)
{
    oracle_b1h(nlev_elem, nl, nEdges, plus, minus, adf_h, edges, edge_tri);
    oracle_b2(nNodes, nlev_nod, nl, plus, minus, area_inv, ttf_max, ttf_min, flux_eps, dt);
}

/*
 * Phase-1 sequencer, header form (include/fesom2-accelerate.h:235 of the reference, 28 args; the
 * reference definition at reference.cpp:289 has 30 and is not exported with C linkage).
 * alg_state 0 -> 1 (a1) -> 2 (a2) -> 4 (a3) -> 5 (a4); vlimit != 1 stops at 2 (reference.cpp:297-303).
 * The oracle additionally runs the Fortran vlimit 2/3 when vlimit_ext != 0 (then alg_state 5 too).
 */
int oracle_pre_comm(double *ttf_max, double *ttf_min, double *plus, double *minus,
                    const double *ttf, const double *LO, const double *adf_v, const double *adf_h,
                    double *UV_rhs, const double *area_inv, int myDim_nod2D, int eDim_nod2D,
                    int myDim_elem2D, int myDim_edge2D, int nl, const int *nlev_nod,
                    const int *nlev_elem, const int *elem2D_nodes, const int *nie_num,
                    const int *nie, int dim, const int *edges, const int *edge_tri, int vlimit,
                    double flux_eps, double big, double dt, int vlimit_ext)
{
    int alg_state = 0;
    oracle_a1(myDim_nod2D + eDim_nod2D, nlev_nod, nl, ttf_max, ttf_min, LO, ttf);
    alg_state = 1;
    oracle_a2(myDim_elem2D, nlev_elem, nl, UV_rhs, elem2D_nodes, ttf_max, ttf_min, big);
    alg_state = 2;
    if (vlimit == 1)
        oracle_a3(myDim_nod2D, nlev_nod, nl, ttf_max, ttf_min, LO, UV_rhs, plus, minus, adf_v,
                  nie, nie_num, dim);
    else if (vlimit_ext && (vlimit == 2 || vlimit == 3))
        oracle_a3_vlimit23(vlimit, myDim_nod2D, nlev_nod, nl, ttf_max, ttf_min, LO, UV_rhs, plus,
                           minus, adf_v, nie, nie_num, dim);
    else
        return alg_state;
    alg_state = 4;
    oracle_a4(myDim_nod2D, nlev_nod, nlev_elem, nl, myDim_edge2D, plus, minus, adf_h, area_inv,
              ttf_max, ttf_min, edges, edge_tri, flux_eps, dt);
    alg_state = 5;
    return alg_state;
}

/* b3-vertical: docs/refactoring.md:204-233, kernels/fct_ale_b3_vertical.cu:2-46.  adf_v2 (iter_yn) may be NULL. */
void oracle_b3v(int nNodes, const int *nlev_nod, int nl, double *adf_v, const double *plus,
                const double *minus, double *adf_v2)
{
    const int L = nl - 1;
    for (int n = 0; n < nNodes; n++) {
        const long b = (long)n * L;
        const long a = (long)n * nl;
        double ae = 1.0;
        double flux = adf_v[a];
        if (flux >= 0.0)
            ae = RMIN(ae, plus[b]);
        else
            ae = RMIN(ae, minus[b]);
        adf_v[a] = ae * adf_v[a];
        for (int z = 1; z < nlev_nod[n] - 1; z++) {
            ae = 1.0;
            flux = adf_v[a + z];
            if (flux >= 0.0) {
                ae = RMIN(ae, minus[b + z - 1]);
                ae = RMIN(ae, plus[b + z]);
            } else {
                ae = RMIN(ae, plus[b + z - 1]);
                ae = RMIN(ae, minus[b + z]);
            }
            if (adf_v2)
                adf_v2[a + z] = (1.0 - ae) * adf_v[a + z];
            adf_v[a + z] = ae * adf_v[a + z];
        }
    }
}

static inline int edge_levels(int e, const int *nlev_elem, const int *edge_tri)
{
    int el1 = edge_tri[2 * e] - 1;
    int el2 = edge_tri[2 * e + 1] - 1;
    int nl1 = nlev_elem[el1] - 1;
    int nl2 = (el2 >= 0) ? (nlev_elem[el2] - 1) : 0;
    return RMAX(nl1, nl2);
}

/* b3-horizontal: docs/refactoring.md:237-263, kernels/fct_ale_b3_horizontal.cu:2-42.  adf_h2 may be NULL. */
void oracle_b3h(int nEdges, const int *nlev_elem, int nl, const int *edges, const int *edge_tri,
                double *adf_h, const double *plus, const double *minus, double *adf_h2)
{
    const int L = nl - 1;
    for (int e = 0; e < nEdges; e++) {
        long n1 = (long)(edges[2 * e] - 1) * L;
        long n2 = (long)(edges[2 * e + 1] - 1) * L;
        int maxLev = edge_levels(e, nlev_elem, edge_tri);
        for (int z = 0; z < maxLev; z++) {
            long i = (long)e * L + z;
            double ae = 1.0;
            double flux = adf_h[i];
            if (flux >= 0.0) {
                ae = RMIN(ae, plus[n1 + z]);
                ae = RMIN(ae, minus[n2 + z]);
            } else {
                ae = RMIN(ae, minus[n1 + z]);
                ae = RMIN(ae, plus[n2 + z]);
            }
            if (adf_h2)
                adf_h2[i] = (1.0 - ae) * adf_h[i];
            adf_h[i] = ae * adf_h[i];
        }
    }
}

/* c-vertical: docs/refactoring.md:295-300 in the order of kernels/fct_ale_c_vertical.cu:9-12 */
void oracle_cv(int nNodes, const int *nlev_nod, int nl, double *del_v, const double *ttf,
               const double *hnode, const double *LO, const double *hnode_new,
               const double *adf_v, double dt, const double *area)
{
    const int L = nl - 1;
    for (int n = 0; n < nNodes; n++)
        for (int z = 0; z < nlev_nod[n] - 1; z++) {
            long i = (long)n * L + z;
            long a = (long)n * nl + z;
            double t = del_v[i] - ttf[i] * hnode[i];
            t = t + LO[i] * hnode_new[i];
            t = t + (adf_v[a] - adf_v[a + 1]) * (dt / area[a]);
            del_v[i] = t;
        }
}

/* c-horizontal: docs/refactoring.md:302-314 in the order of kernels/fct_ale_c_horizontal.cu:22-26 */
void oracle_ch(int nEdges, const int *nlev_elem, int nl, const int *edges, const int *edge_tri,
               double *del_h, const double *adf_h, double dt, const double *area)
{
    const int L = nl - 1;
    for (int e = 0; e < nEdges; e++) {
        int n1 = edges[2 * e] - 1;
        int n2 = edges[2 * e + 1] - 1;
        int maxLev = edge_levels(e, nlev_elem, edge_tri);
        for (int z = 0; z < maxLev; z++) {
            double a = adf_h[(long)e * L + z];
            del_h[(long)n1 * L + z] = del_h[(long)n1 * L + z] + a * (dt / area[(long)n1 * nl + z]);
            del_h[(long)n2 * L + z] = del_h[(long)n2 * L + z] - a * (dt / area[(long)n2 * nl + z]);
        }
    }
}

/*
 * iter_yn "update the LO" branch: docs/refactoring.md:265-290.  Fortran order
 * LO + (adf_v[z]-adf_v[z+1])*dt/area/hnode_new, i.e. (((d*dt)/area)/hnode_new), and
 * LO(n1) + adf_h*dt/area/hnode_new, LO(n2) - adf_h*dt/area/hnode_new.
 * After it the Fortran swaps adf <- adf2 (the caller does the swap).
 */
void oracle_lo_update(int nNodes, const int *nlev_nod, int nEdges, const int *nlev_elem, int nl,
                      const int *edges, const int *edge_tri, double *LO, const double *adf_v,
                      const double *adf_h, double dt, const double *area, const double *hnode_new)
{
    const int L = nl - 1;
    for (int n = 0; n < nNodes; n++)
        for (int z = 0; z < nlev_nod[n] - 1; z++) {
            long i = (long)n * L + z;
            long a = (long)n * nl + z;
            LO[i] = LO[i] + (adf_v[a] - adf_v[a + 1]) * dt / area[a] / hnode_new[i];
        }
    for (int e = 0; e < nEdges; e++) {
        int n1 = edges[2 * e] - 1;
        int n2 = edges[2 * e + 1] - 1;
        int maxLev = edge_levels(e, nlev_elem, edge_tri);
        for (int z = 0; z < maxLev; z++) {
            double a = adf_h[(long)e * L + z];
            long i1 = (long)n1 * L + z, i2 = (long)n2 * L + z;
            LO[i1] = LO[i1] + a * dt / area[(long)n1 * nl + z] / hnode_new[i1];
            LO[i2] = LO[i2] - a * dt / area[(long)n2 * nl + z] / hnode_new[i2];
        }
    }
}

/*
 * Whole non-iterative pass on one domain (no halo exchange needed when eDim_nod2D == 0):
 * pre_comm (a1..b2) -> b3v -> b3h -> cv -> ch.  Returns the last alg_state (5 on success).
 */
int oracle_full_pass(double *ttf_max, double *ttf_min, double *plus, double *minus,
                     const double *ttf, const double *LO, double *adf_v, double *adf_h,
                     double *UV_rhs, const double *area, const double *area_inv,
                     const double *hnode, const double *hnode_new, double *del_v, double *del_h,
                     int myDim_nod2D, int eDim_nod2D, int myDim_elem2D, int myDim_edge2D, int nl,
                     const int *nlev_nod, const int *nlev_elem, const int *elem2D_nodes,
                     const int *nie_num, const int *nie, int dim, const int *edges,
                     const int *edge_tri, int vlimit, double flux_eps, double big, double dt)
{
    int st = oracle_pre_comm(ttf_max, ttf_min, plus, minus, ttf, LO, adf_v, adf_h, UV_rhs,
                             area_inv, myDim_nod2D, eDim_nod2D, myDim_elem2D, myDim_edge2D, nl,
                             nlev_nod, nlev_elem, elem2D_nodes, nie_num, nie, dim, edges, edge_tri,
                             vlimit, flux_eps, big, dt, 1);
    if (st != 5)
        return st;
    oracle_b3v(myDim_nod2D, nlev_nod, nl, adf_v, plus, minus, NULL);
    oracle_b3h(myDim_edge2D, nlev_elem, nl, edges, edge_tri, adf_h, plus, minus, NULL);
    oracle_cv(myDim_nod2D, nlev_nod, nl, del_v, ttf, hnode, LO, hnode_new, adf_v, dt, area);
    oracle_ch(myDim_edge2D, nlev_elem, nl, edges, edge_tri, del_h, adf_h, dt, area);
    return st;
}
