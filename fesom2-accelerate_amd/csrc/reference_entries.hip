// reference_entries.hip -- the reference's CPU-named entry points, executed by the GPU engine.
//
// The reference header exports fct_ale_a1_reference_ .. fct_ale_a4_reference_ and
// fct_ale_pre_comm_ (include/fesom2-accelerate.h:142, :225-235; src/reference.cpp:289-438) on host
// arrays.  A drop-in library must keep those symbols and their meaning, so they are provided here
// with the same arguments -- but the arithmetic runs in the HIP kernels: stage the host arrays,
// launch, copy the results back (synchronous, null stream).  The sizes the reference never passes
// (how many node columns a2/a4 touch, how many element columns a3 reads) are derived from the
// connectivity, and every index is validated before anything is launched.
#include "f2a_host.hpp"

#include <algorithm>
#include <vector>

using namespace f2a;

namespace {

struct Staged {
    std::vector<void *> ptrs;
    ~Staged()
    {
        for (void *p : ptrs) (void)hipFree(p);
    }
    template <class T>
    T *put(const T *host, size_t n)
    {
        void *p = nullptr;
        if (!ok(hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T) + kAllocPad), "hipMalloc(staging)")) return nullptr;  // + pad: ldo
        ptrs.push_back(p);
        if (host && n && !ok(hipMemcpy(p, host, n * sizeof(T), hipMemcpyHostToDevice), "H2D(staging)")) return nullptr;
        return static_cast<T *>(p);
    }
};

template <class T>
bool get(T *host, const T *dev, size_t n)
{
    return !n || ok(hipMemcpy(host, dev, n * sizeof(T), hipMemcpyDeviceToHost), "D2H(staging)");
}

bool levels_ok(const int *nlev, long n, int nl, const char *who)
{
    for (long i = 0; i < n; i++)
        if (nlev[i] < 1 || nlev[i] > nl) {
            report("%s: nlevels(%ld) = %d outside 1..%d", who, i + 1, nlev[i], nl);
            return false;
        }
    return true;
}

long max_index(const int *a, size_t n)
{
    long m = 0;
    for (size_t i = 0; i < n; i++) m = std::max<long>(m, a[i]);
    return m;
}

bool positive(const int *a, size_t n, const char *who)
{
    for (size_t i = 0; i < n; i++)
        if (a[i] < 1) {
            report("%s: entry %zu = %d (1-based index expected)", who, i + 1, a[i]);
            return false;
        }
    return true;
}

}  // namespace

extern "C" {

void fct_ale_a1_reference_(int *nNodes, int *nLevels_nod2D, int *nl, real *fct_ttf_max,
                           real *fct_ttf_min, real *fct_low_order, real *ttf)
{
    const long n = *nNodes;
    const int L = *nl - 1;
    if (n <= 0 || !check_levels(*nl, "fct_ale_a1_reference_") || !levels_ok(nLevels_nod2D, n, *nl, "fct_ale_a1_reference_"))
        return;
    Staged s;
    const size_t c = (size_t)n * L;
    int *lev = s.put(nLevels_nod2D, n);
    real *lo = s.put(fct_low_order, c), *t = s.put(ttf, c), *mx = s.put(fct_ttf_max, c), *mn = s.put(fct_ttf_min, c);
    if (!lev || !lo || !t || !mx || !mn) return;
    if (!ok(launch_a1((int)n, *nl, lev, lo, t, mx, mn, nullptr), "fct_ale_a1")) return;
    get(fct_ttf_max, mx, c) && get(fct_ttf_min, mn, c);
}

void fct_ale_a2_reference_(int *nElements, int *nLevels_elem2D, int *nl, real *UV_rhs,
                           int *elem2D_nodes, real *fct_ttf_max, real *fct_ttf_min, real *bignumber)
{
    const long T = *nElements;
    const int L = *nl - 1;
    if (T <= 0 || !check_levels(*nl, "fct_ale_a2_reference_") || !levels_ok(nLevels_elem2D, T, *nl, "fct_ale_a2_reference_") ||
        !positive(elem2D_nodes, 3 * (size_t)T, "fct_ale_a2_reference_ elem2D_nodes"))
        return;
    const long nn = max_index(elem2D_nodes, 3 * (size_t)T);
    Staged s;
    int *lev = s.put(nLevels_elem2D, T), *en = s.put(elem2D_nodes, 3 * (size_t)T);
    real *mx = s.put(fct_ttf_max, (size_t)nn * L), *mn = s.put(fct_ttf_min, (size_t)nn * L);
    real *uv = s.put<real>(nullptr, 2 * (size_t)L * T);
    if (!lev || !en || !mx || !mn || !uv) return;
    if (!ok(launch_a2((int)T, *nl, lev, en, mx, mn, uv, *bignumber, nullptr), "fct_ale_a2")) return;
    get(UV_rhs, uv, 2 * (size_t)L * T);
}

void fct_ale_a3_reference_(int *nNodes2D, int *nLevels_nod2D, int *nl, real *fct_ttf_max,
                           real *fct_ttf_min, real *fct_LO, real *UV_rhs, real *fct_plus,
                           real *fct_minus, real *fct_adf_v, int *nod_in_elem2D,
                           int *nod_in_elem2D_num, int *nod_in_elem2D_dim)
{
    const long n = *nNodes2D;
    const int L = *nl - 1, dim = *nod_in_elem2D_dim;
    if (n <= 0 || dim < 1 || !check_levels(*nl, "fct_ale_a3_reference_") ||
        !levels_ok(nLevels_nod2D, n, *nl, "fct_ale_a3_reference_"))
        return;
    long ne = 0;
    for (long i = 0; i < n; i++) {
        if (nod_in_elem2D_num[i] < 1 || nod_in_elem2D_num[i] > dim) {
            report("fct_ale_a3_reference_: nod_in_elem2D_num(%ld) = %d outside 1..%d", i + 1, nod_in_elem2D_num[i], dim);
            return;
        }
        if (!positive(nod_in_elem2D + i * dim, nod_in_elem2D_num[i], "fct_ale_a3_reference_ nod_in_elem2D")) return;
        ne = std::max(ne, max_index(nod_in_elem2D + i * dim, nod_in_elem2D_num[i]));
    }
    Staged s;
    const size_t c = (size_t)n * L;
    int *lev = s.put(nLevels_nod2D, n), *nie = s.put(nod_in_elem2D, (size_t)n * dim), *num = s.put(nod_in_elem2D_num, n);
    real *mx = s.put(fct_ttf_max, c), *mn = s.put(fct_ttf_min, c), *lo = s.put(fct_LO, c);
    real *uv = s.put(UV_rhs, 2 * (size_t)L * ne), *p = s.put(fct_plus, c), *m = s.put(fct_minus, c);
    real *av = s.put(fct_adf_v, (size_t)n * *nl);
    if (!lev || !nie || !num || !mx || !mn || !lo || !uv || !p || !m || !av) return;
    if (!ok(launch_a3((int)n, *nl, 1, lev, nie, num, dim, uv, lo, mx, mn, nullptr), "fct_ale_a3")) return;
    if (!ok(launch_b1v((int)n, *nl, lev, av, p, m, nullptr), "fct_ale_b1_vertical")) return;
    get(fct_ttf_max, mx, c) && get(fct_ttf_min, mn, c) && get(fct_plus, p, c) && get(fct_minus, m, c);
}

void fct_ale_a4_reference_(int *nNodes2D, int *nLevels_nod2D, int *nLevels_elem2D, int *nl,
                           int *nEdges2D, real *fct_plus, real *fct_minus, real *fct_adf_h,
                           real *area_inv, real *fct_ttf_max, real *fct_ttf_min, int *edges,
                           int *edge_tri, real *flux_eps, real *dt)
{
    const long n = *nNodes2D, E = *nEdges2D;
    const int L = *nl - 1;
    if (n < 0 || E < 0 || !check_levels(*nl, "fct_ale_a4_reference_") ||
        !levels_ok(nLevels_nod2D, n, *nl, "fct_ale_a4_reference_") ||
        !positive(edges, 2 * (size_t)E, "fct_ale_a4_reference_ edges"))
        return;
    for (long e = 0; e < E; e++)
        if (edge_tri[2 * e] < 1 || edge_tri[2 * e + 1] < 0) {
            report("fct_ale_a4_reference_: edge_tri(:,%ld) = (%d,%d)", e + 1, edge_tri[2 * e], edge_tri[2 * e + 1]);
            return;
        }
    // b1-horizontal adds into every node an edge touches (halo included), like reference.cpp:406-425
    const long nn = std::max<long>(n, max_index(edges, 2 * (size_t)E));
    const long ne = max_index(edge_tri, 2 * (size_t)E);
    if (!levels_ok(nLevels_elem2D, ne, *nl, "fct_ale_a4_reference_ (elements)")) return;
    HostMesh hm;
    hm.edges = edges;
    hm.edge_tri = edge_tri;
    hm.nlev_elem = nLevels_elem2D;
    hm.n_elem_total = ne;
    std::string err;
    auto plan = build_plan(hm, (int)nn, (int)nn, (int)E, (int)nn, *nl, PlanShape{}, err);
    if (!plan) {
        report("fct_ale_a4_reference_: invalid mesh: %s", err.c_str());
        return;
    }
    Staged s;
    int *lev = s.put(nLevels_nod2D, n);
    real *p = s.put(fct_plus, (size_t)nn * L), *m = s.put(fct_minus, (size_t)nn * L), *ah = s.put(fct_adf_h, (size_t)E * L);
    real *ai = s.put(area_inv, (size_t)n * *nl), *mx = s.put(fct_ttf_max, (size_t)n * L), *mn = s.put(fct_ttf_min, (size_t)n * L);
    if (!lev || !p || !m || !ah || !ai || !mx || !mn) return;
    if (!ok(launch_b1h(plan->dev, *nl, ah, p, m, nullptr), "fct_ale_b1_horizontal")) return;
    if (!ok(launch_b2((int)n, *nl, lev, ai, mx, mn, p, m, *dt, *flux_eps, nullptr), "fct_ale_b2")) return;
    get(fct_plus, p, (size_t)nn * L) && get(fct_minus, m, (size_t)nn * L);
}

// Header form (28 arguments) of the reference's sequencer, src/reference.cpp:289-304: a1 on owned +
// halo nodes, a2, and for vlimit == 1 a3 and a4; alg_state 0 -> 1 -> 2 -> 4 -> 5.
void fct_ale_pre_comm_(int *alg_state, real *fct_ttf_max, real *fct_ttf_min, real *fct_plus,
                       real *fct_minus, real *ttf, real *fct_LO, real *fct_adf_v, real *fct_adf_h,
                       real *UV_rhs, real *area_inv, int *myDim_nod2D, int *eDim_nod2D,
                       int *myDim_elem2D, int *myDim_edge2D, int *nl, int *nlevels_nod2D,
                       int *nlevels_elem2D, int *elem2D_nodes, int *nod_in_elem2D_num,
                       int *nod_in_elem2D, int *nod_in_elem2D_dim, int *nod2D_edges,
                       int *elem2D_edges, int *vlimit, real *flux_eps, real *bignumber, real *dt)
{
    *alg_state = 0;
    int nNodes = *myDim_nod2D + *eDim_nod2D;
    const unsigned long nerr = error_count();
    auto failed = [&] { return error_count() != nerr; };
    fct_ale_a1_reference_(&nNodes, nlevels_nod2D, nl, fct_ttf_max, fct_ttf_min, fct_LO, ttf);
    if (failed()) return;
    *alg_state = 1;
    fct_ale_a2_reference_(myDim_elem2D, nlevels_elem2D, nl, UV_rhs, elem2D_nodes, fct_ttf_max, fct_ttf_min, bignumber);
    if (failed()) return;
    *alg_state = 2;
    if (*vlimit == 1) {
        fct_ale_a3_reference_(myDim_nod2D, nlevels_nod2D, nl, fct_ttf_max, fct_ttf_min, fct_LO, UV_rhs, fct_plus,
                              fct_minus, fct_adf_v, nod_in_elem2D, nod_in_elem2D_num, nod_in_elem2D_dim);
        if (failed()) return;
        *alg_state = 4;
        fct_ale_a4_reference_(myDim_nod2D, nlevels_nod2D, nlevels_elem2D, nl, myDim_edge2D, fct_plus, fct_minus,
                              fct_adf_h, area_inv, fct_ttf_max, fct_ttf_min, nod2D_edges, elem2D_edges, flux_eps, dt);
        if (failed()) return;
        *alg_state = 5;
    }
}

}  // extern "C"
