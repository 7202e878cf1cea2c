// fesom2_accelerate.hip -- the C-ABI of libfesom2-accelerate.so: memory/stream entry points and the
// FCT-ALE phases.
//
// Mirrors the reference's host layer (src/fesom2-accelerate.cu:17-379): opaque buffer handles,
// streams and events, and the three phase entry points around the MPI halo exchange, plus the
// additions declared in include/fesom2-accelerate.h (c-step, fused phase 2, resident mode).
// Unlike the reference it validates every handle and mesh index on the host before a kernel can
// touch it, checks every launch, and never computes anything on the CPU.
#include "f2a_host.hpp"

#include <cstdio>
#include <cstdlib>
#include <initializer_list>

using namespace f2a;


extern "C" {

void set_mpi_rank_(int *rank, int *total_ranks)
{
    // reference src/fesom2-accelerate.cu:206-228
    const int rank_on_node = (*total_ranks > 0) ? (*rank) % (*total_ranks) : *rank;
    int count = 0;
    if (!ok(hipGetDeviceCount(&count), "hipGetDeviceCount")) return;
    if (count < 1) {
        report("no HIP devices found on the node where rank %d runs", *rank);
        return;
    }
    const int dev = rank_on_node % count;
    if (!ok(hipSetDevice(dev), "hipSetDevice")) report("error in setting device id to %d", dev);
}

void transfer_mesh_(void **ret, int *host_ptr, int *size, int *istat)
{
    if (*size < 0) {
        report("transfer_mesh_: size %d < 0", *size);
        *ret = nullptr;
        *istat = 1;
        return;
    }
    Buffer *m = allocate(host_ptr, (size_t)(*size) * sizeof(int), false);
    if (m && h2d(m, true, nullptr, false)) {
        *ret = m;
        *istat = 0;
    } else {
        *ret = nullptr;
        *istat = 1;
    }
}

static void alloc_doubles(void **ret, real *host_ptr, long long n, bool *create_event, int *istat, const char *who)
{
    *ret = nullptr;
    *istat = 1;
    if (n < 0) {
        report("%s: size %lld < 0 (arrays of 2^31 or more doubles need fesom2_alloc_var_i8_)", who, n);
        return;
    }
    Buffer *m = allocate(host_ptr, (size_t)n * sizeof(real), create_event && *create_event);
    *istat = m ? 0 : 1;
    *ret = m;
}

void alloc_var_(void **ret, real *host_ptr, int *size, bool *create_event, int *istat)
{
    alloc_doubles(ret, host_ptr, *size, create_event, istat, "alloc_var_");
}

void reserve_var_(void **ret, int *size, bool *create_event, int *istat)
{
    alloc_doubles(ret, nullptr, *size, create_event, istat, "reserve_var_");
}

// 64-bit sizes: a whole 9.6M x 80 mesh on one GPU has 2.3e9-element fct_adf_h (the reference's
// int size stops at 2^31-1)
void fesom2_alloc_var_i8_(void **ret, real *host_ptr, long long *size, bool *create_event, int *istat)
{
    alloc_doubles(ret, host_ptr, *size, create_event, istat, "fesom2_alloc_var_i8_");
}

void fesom2_reserve_var_i8_(void **ret, long long *size, bool *create_event, int *istat)
{
    alloc_doubles(ret, nullptr, *size, create_event, istat, "fesom2_reserve_var_i8_");
}

void allocate_pinned_doubles_(void **hostptr, int *size, int *istat)
{
    *istat = 0;
    if (!ok(hipHostMalloc(hostptr, sizeof(real) * (size_t)(*size), hipHostMallocDefault), "hipHostMalloc")) {
        fprintf(stderr, "fesom2-accelerate: error in allocating page-locked memory, using normal malloc...\n");
        *hostptr = malloc(sizeof(real) * (size_t)(*size));
        *istat = 1;
    }
}

void transfer_var_(void **mem, real *host_ptr)
{
    Buffer *b = buf(mem, "transfer_var_");
    if (!b) return;
    mark_internal(b, nullptr, nullptr);  // new raw contents
    b->host_pointer = host_ptr;
    h2d(b, true, nullptr, false);
}

void transfer_var_async_(void **mem, real *host_ptr, void **stream, bool *record_event)
{
    Buffer *b = buf(mem, "transfer_var_async_");
    if (!b) return;
    mark_internal(b, nullptr, stream_of(stream));
    b->host_pointer = host_ptr;
    h2d(b, false, stream_of(stream), record_event && *record_event);
}

void fesom2_transfer_back_async_(void **mem, real *host_ptr, void **stream, int *istat)
{
    *istat = 1;
    Buffer *b = buf(mem, "fesom2_transfer_back_async_");
    if (!b) return;
    if (!host_ptr) {
        report("fesom2_transfer_back_async_: no host array");
        return;
    }
    b->host_pointer = host_ptr;
    if (d2h_async(b, stream_of(stream))) *istat = 0;
}

void make_stream_(void **stream, int *istat)
{
    *istat = 0;
    auto *s = new hipStream_t;
    if (!ok(hipStreamCreate(s), "hipStreamCreate")) {
        *istat = 1;
        fprintf(stderr, "fesom2-accelerate: error in creating HIP stream... returning default stream\n");
        *s = nullptr;
    }
    *stream = s;
}

void await_stream_(void **s, int *istat)
{
    *istat = ok(hipStreamSynchronize(stream_of(s)), "hipStreamSynchronize") ? 0 : 1;
}

// ----------------------------------------------------------------------------- phase 1

}  // extern "C"

// The c-vertical fields bound to fct_adf_v (fesom2_bind_c_vertical_), checked alive and large
// enough for N owned columns; out[] stays null when nothing is bound.  false (reported) on a stale
// or short binding.
static bool bound_c_vertical(Buffer *adf_v, int N, int L, int NL, Buffer *out[4])
{
    const CvBinding *cv = adf_v->cv;
    if (!cv) return true;
    for (int k = 0; k < 4; k++)
        if (!object_live(cv->b[k], cv->serial[k])) {
            report("fesom2_bind_c_vertical_: a bound field was freed (bind again)");
            return false;
        }
    const size_t need[4] = {col_bytes(N, L), col_bytes(N, L), col_bytes(N, L), col_bytes(N, NL)};
    for (int k = 0; k < 4; k++)
        if (cv->b[k]->size < need[k]) {
            report("fesom2_bind_c_vertical_: a bound field holds %zu bytes, %zu needed", cv->b[k]->size, need[k]);
            return false;
        }
    for (int k = 0; k < 4; k++) out[k] = cv->b[k];
    return true;
}

extern "C" {

void fesom2_bind_c_vertical_(int *istat, void **fct_adf_v, void **del_ttf_advvert, void **hnode, void **hnode_new,
                             void **area)
{
    *istat = 1;
    Buffer *bv = buf(fct_adf_v, "fct_adf_v");
    if (!bv) return;
    void **hs[4] = {del_ttf_advvert, hnode, hnode_new, area};
    const bool unbind = !(del_ttf_advvert && *del_ttf_advvert) && !(hnode && *hnode) &&
                        !(hnode_new && *hnode_new) && !(area && *area);
    if (unbind) {
        delete bv->cv;
        bv->cv = nullptr;
        *istat = 0;
        return;
    }
    static const char *names[4] = {"del_ttf_advvert", "hnode", "hnode_new", "area"};
    auto *cv = new CvBinding;
    for (int k = 0; k < 4; k++) {
        cv->b[k] = buf(hs[k], names[k]);
        if (!cv->b[k]) {
            delete cv;
            return;
        }
        cv->serial[k] = cv->b[k]->serial;
    }
    delete bv->cv;
    bv->cv = cv;
    *istat = 0;
}


void fct_ale_pre_comm_acc_(int *alg_state, void **s, void **fct_ttf_max, void **fct_ttf_min,
                           void **fct_plus, void **fct_minus, void **ttf, void **fct_LO,
                           void **fct_adf_v, void **fct_adf_h, void **UV_rhs, void **area_inv,
                           int *myDim_nod2D, int *eDim_nod2D, int *myDim_elem2D, int *myDim_edge2D,
                           int *nl, void **nlevels_nod2D, void **nlevels_elem2D, void **elem2D_nodes,
                           void **nod_in_elem2D_num, void **nod_in_elem2D, int *nod_in_elem2D_dim,
                           void **nod2D_edges, void **elem2D_edges, int *vlimit, real *flux_eps,
                           real *bignumber, real *dt)
{
    const PhaseRange range("fct_ale_pre_comm_acc_");
    *alg_state = 0;
    const hipStream_t st = stream_of(s);
    const int N = *myDim_nod2D, NT = *myDim_nod2D + *eDim_nod2D, T = *myDim_elem2D, E = *myDim_edge2D;
    const int NL = *nl, L = NL - 1;
    if (!check_levels(NL, "fct_ale_pre_comm_acc_")) return;
    MeshHandles mh;
    mh.edges = need(nod2D_edges, 2 * sizeof(int) * (size_t)E, "nod2D_edges");
    mh.edge_tri = need(elem2D_edges, 2 * sizeof(int) * (size_t)E, "elem2D_edges");
    mh.nlev_elem = need(nlevels_elem2D, sizeof(int) * (size_t)T, "nlevels_elem2D");
    Buffer *bnlnod = need(nlevels_nod2D, sizeof(int) * (size_t)NT, "nlevels_nod2D");
    mh.elem_nodes = need(elem2D_nodes, 3 * sizeof(int) * (size_t)T, "elem2D_nodes");
    mh.nie = buf(nod_in_elem2D, "nod_in_elem2D");
    mh.nie_num = buf(nod_in_elem2D_num, "nod_in_elem2D_num");
    mh.dim = *nod_in_elem2D_dim;
    Buffer *bmax = buf(fct_ttf_max, "fct_ttf_max"), *bmin = buf(fct_ttf_min, "fct_ttf_min");
    Buffer *bplus = need(fct_plus, col_bytes(N, L), "fct_plus");
    Buffer *bminus = need(fct_minus, col_bytes(N, L), "fct_minus");
    Buffer *bttf = need(ttf, col_bytes(NT, L), "ttf");
    Buffer *blo = need(fct_LO, col_bytes(NT, L), "fct_LO");
    Buffer *badfv = need(fct_adf_v, col_bytes(N, NL), "fct_adf_v");
    Buffer *badfh = need(fct_adf_h, col_bytes(E, L), "fct_adf_h");
    Buffer *buv = buf(UV_rhs, "UV_rhs");
    Buffer *bainv = need(area_inv, col_bytes(N, NL), "area_inv");
    if (!mh.edges || !mh.edge_tri || !mh.nlev_elem || !bnlnod || !mh.elem_nodes || !mh.nie ||
        !mh.nie_num || !bmax || !bmin || !bplus || !bminus || !bttf || !blo || !badfv || !badfh ||
        !buv || !bainv)
        return;
    const bool stepwise = kernel_path() == 1;
    mh.nlev_nod = bnlnod;
    const Plan *plan = get_plan(mh, N, NT, E, NL, !stepwise);
    if (!plan) return;

    if (!g_resident && !h2d(blo, false, st, false)) return;  // reference :268
    const int *nlev_nod = dptr<int>(bnlnod);
    wait_event(bttf, st);  // reference :293 ("ttf: transferred before fct_ale_muscl_LH")
    wait_event(badfv, st);
    wait_event(badfh, st);

    auto finish = [&](int state, std::initializer_list<Buffer *> outs) {
        *alg_state = state;
        if (!g_resident)
            for (Buffer *b : outs)
                if (!d2h_async(b, st)) {
                    *alg_state = 0;  // reference transfer_back :249-253
                    return;
                }
    };

    // every path: fluxes a phase-1 call already limited in part (fast mode, pre_comm_v) are refused
    if (has_internal(badfv, st) || has_internal(badfh, st)) {
        report("fct_ale_pre_comm_acc_: fct_adf_v/fct_adf_h already hold a limited phase 2 part (upload "
               "the raw fluxes first)");
        return;
    }
    if (!stepwise) {
        f2a::P1Args a{N, NL, *vlimit, nlev_nod, dptr<real>(bttf), dptr<real>(blo), dptr<real>(badfv),
                      dptr<real>(badfh), dptr<real>(bainv), dptr<real>(bplus), dptr<real>(bminus),
                      *dt, *flux_eps, *bignumber};
        a.tr.order = f2a::pass_order(*plan, 1);  // kernel directions (Infinity Cache reuse)
        if (kernel_path() == 2) {
            // fast mode: b3-vertical (and the block-internal edges' b3-horizontal) while the block's
            // plus/minus are in LDS; inter_comm / post_comm find the marks and do the rest
            Buffer *cvb[4] = {nullptr, nullptr, nullptr, nullptr};
            if (!bound_c_vertical(badfv, N, L, NL, cvb)) return;
            if (cvb[0]) {  // c-vertical too (fesom2_bind_c_vertical_)
                if (has_internal(cvb[0], st)) {
                    report("fct_ale_pre_comm_acc_: the bound del_ttf_advvert already holds this pass's c-vertical");
                    return;
                }
                a.del_v = dptr<real>(cvb[0]);
                a.hnode = dptr<real>(cvb[1]);
                a.hnode_new = dptr<real>(cvb[2]);
                a.area = dptr<real>(cvb[3]);
                if (!run("fct_ale_p1v", st, [&] { return f2a::launch_p1v(plan->dev, a, st); })) return;
                mark_internal(cvb[0], plan, st);
            } else if (!run("fct_ale_p1_b3v", st, [&] { return f2a::launch_p1_b3v(plan->dev, a, st); })) {
                return;
            }
            mark_internal(badfv, plan, st);
            mark_internal(badfh, f2a::p1v_limits_internal(plan->dev, a) ? plan : nullptr, st);
        } else if (!run("fct_ale_p1", st, [&] { return f2a::launch_p1_fused(plan->dev, a, st); })) {
            return;
        }
        finish(6, {bplus, bminus});
        return;
    }

    // stepwise path: one kernel per reference step, reference alg_state numbering (:294-337)
    if (!need(fct_ttf_max, col_bytes(NT, L), "fct_ttf_max") || !need(fct_ttf_min, col_bytes(NT, L), "fct_ttf_min") ||
        !need(UV_rhs, col_bytes(T, 2 * L), "UV_rhs") || mh.nie->size < sizeof(int) * (size_t)mh.dim * N ||
        mh.nie_num->size < sizeof(int) * (size_t)N) {
        report("fct_ale_pre_comm_acc_: scratch or nod_in_elem2D handles too small");
        return;
    }
    const int limit = plan->num_kernels;
    real *tmax = dptr<real>(bmax), *tmin = dptr<real>(bmin);
    if (!run("fct_ale_a1", st, [&] { return f2a::launch_a1(NT, NL, nlev_nod, dptr<real>(blo), dptr<real>(bttf), tmax, tmin, st); })) return;
    if (limit < 2) return finish(1, {bmax, bmin});
    if (!run("fct_ale_a2", st, [&] { return f2a::launch_a2(T, NL, dptr<int>(mh.nlev_elem), dptr<int>(mh.elem_nodes), tmax, tmin, dptr<real>(buv), *bignumber, st); }))
        return;
    if (limit < 3) return finish(2, {bmax, bmin, buv});
    if (!run("fct_ale_a3", st, [&] { return f2a::launch_a3(N, NL, *vlimit, nlev_nod, dptr<int>(mh.nie), dptr<int>(mh.nie_num), mh.dim,
                           dptr<real>(buv), dptr<real>(blo), tmax, tmin, st); }))
        return;
    if (limit < 4) return finish(3, {bmax, bmin});
    if (!run("fct_ale_b1_vertical", st, [&] { return f2a::launch_b1v(N, NL, nlev_nod, dptr<real>(badfv), dptr<real>(bplus), dptr<real>(bminus), st); }))
        return;
    if (limit < 5) return finish(4, {bmax, bmin, bplus, bminus});
    if (!run("fct_ale_b1_horizontal", st, [&] { return f2a::launch_b1h(plan->dev, NL, dptr<real>(badfh), dptr<real>(bplus), dptr<real>(bminus), st); }))
        return;
    if (limit < 6) return finish(5, {bmax, bmin, bplus, bminus});
    if (!run("fct_ale_b2", st, [&] { return f2a::launch_b2(N, NL, nlev_nod, dptr<real>(bainv), tmax, tmin, dptr<real>(bplus), dptr<real>(bminus), *dt, *flux_eps, st); }))
        return;
    finish(6, {bplus, bminus});
}

// Batched phase 1 (a1..b2, fused) of ntracers tracers in one launch: per-tracer handles hold the
// tracers one after another, (N+H)*L doubles apart (ttf, fct_LO, fct_plus, fct_minus), (N+H)*nl
// apart (fct_adf_v) and E*L apart (fct_adf_h); area_inv is shared.  alg_state 6 on success.
// Fused phase 1 of ntracers tracers; with `area` given (vertical = true) also b3v + cv on the own
// columns (launch_p1v: fct_adf_v limited in place, del_ttf_advvert updated; alg_state 7).
static void pre_comm_fused_impl(int *alg_state, void **s, int *ntracers, void **fct_plus, void **fct_minus,
                                void **ttf, void **fct_LO, void **fct_adf_v, void **fct_adf_h, void **area_inv,
                                int *myDim_nod2D, int *eDim_nod2D, int *myDim_elem2D, int *myDim_edge2D, int *nl,
                                void **nlevels_nod2D, void **nlevels_elem2D, void **elem2D_nodes,
                                void **nod_in_elem2D_num, void **nod_in_elem2D, int *nod_in_elem2D_dim,
                                void **nod2D_edges, void **elem2D_edges, int *vlimit, real *flux_eps,
                                real *bignumber, real *dt, void **area, void **hnode, void **hnode_new,
                                void **del_ttf_advvert, const char *who)
{
    const PhaseRange range(who);
    const bool vertical = area != nullptr;
    *alg_state = 0;
    const hipStream_t st = stream_of(s);
    const int N = *myDim_nod2D, NT = *myDim_nod2D + *eDim_nod2D, T = *myDim_elem2D, E = *myDim_edge2D;
    const int NL = *nl, L = NL - 1, ntr = *ntracers;
    if (!check_levels(NL, who)) return;
    if (ntr < 1) {
        report("%s: ntracers = %d", who, ntr);
        return;
    }
    MeshHandles mh;
    mh.edges = need(nod2D_edges, 2 * sizeof(int) * (size_t)E, "nod2D_edges");
    mh.edge_tri = need(elem2D_edges, 2 * sizeof(int) * (size_t)E, "elem2D_edges");
    mh.nlev_elem = need(nlevels_elem2D, sizeof(int) * (size_t)T, "nlevels_elem2D");
    Buffer *bnlnod = need(nlevels_nod2D, sizeof(int) * (size_t)NT, "nlevels_nod2D");
    mh.elem_nodes = need(elem2D_nodes, 3 * sizeof(int) * (size_t)T, "elem2D_nodes");
    mh.nie = buf(nod_in_elem2D, "nod_in_elem2D");
    mh.nie_num = buf(nod_in_elem2D_num, "nod_in_elem2D_num");
    mh.dim = *nod_in_elem2D_dim;
    const size_t nodeb = col_bytes(NT, L) * ntr;
    Buffer *bplus = need(fct_plus, nodeb, "fct_plus"), *bminus = need(fct_minus, nodeb, "fct_minus");
    Buffer *bttf = need(ttf, nodeb, "ttf"), *blo = need(fct_LO, nodeb, "fct_LO");
    Buffer *badfv = need(fct_adf_v, col_bytes(NT, NL) * ntr, "fct_adf_v");
    Buffer *badfh = need(fct_adf_h, col_bytes(E, L) * ntr, "fct_adf_h");
    Buffer *bainv = need(area_inv, col_bytes(N, NL), "area_inv");
    if (!mh.edges || !mh.edge_tri || !mh.nlev_elem || !bnlnod || !mh.elem_nodes || !mh.nie || !mh.nie_num ||
        !bplus || !bminus || !bttf || !blo || !badfv || !badfh || !bainv)
        return;
    Buffer *barea = nullptr, *bh = nullptr, *bhn = nullptr, *bdv = nullptr;
    if (vertical) {
        barea = need(area, col_bytes(N, NL), "area");
        bh = need(hnode, col_bytes(N, L), "hnode");
        bhn = need(hnode_new, col_bytes(N, L), "hnode_new");
        bdv = need(del_ttf_advvert, ntr > 1 ? nodeb : col_bytes(N, L), "del_ttf_advvert");
        if (!barea || !bh || !bhn || !bdv) return;
    }
    mh.nlev_nod = bnlnod;
    // fluxes a fast-mode fct_ale_pre_comm_acc_ (or an unfinished pre_comm_v) already limited in part:
    // limiting them again would be wrong -- the same guard as the fast mode's own
    if (has_internal(badfv, st) || has_internal(badfh, st) || (bdv && has_internal(bdv, st))) {
        report("%s: fct_adf_v/fct_adf_h/del_ttf_advvert already hold a limited phase 2 part (finish that "
               "phase, or upload the raw fluxes first)", who);
        return;
    }
    const Plan *plan = get_plan(mh, N, NT, E, NL, true, ntr > 1);
    if (!plan) return;
    if (!g_resident && !h2d(blo, false, st, false)) return;
    wait_event(bttf, st);
    wait_event(badfv, st);
    wait_event(badfh, st);
    f2a::P1Args a{N, NL, *vlimit, dptr<int>(bnlnod), dptr<real>(bttf), dptr<real>(blo), dptr<real>(badfv),
                  dptr<real>(badfh), dptr<real>(bainv), dptr<real>(bplus), dptr<real>(bminus),
                  *dt, *flux_eps, *bignumber};
    a.tr = f2a::Tracers{ntr, (size_t)NT * L, (size_t)NT * NL, (size_t)E * L};
    a.tr.order = f2a::pass_order(*plan, ntr);  // kernel directions (Infinity Cache reuse)
    if (vertical) {
        a.area = dptr<real>(barea);
        a.hnode = dptr<real>(bh);
        a.hnode_new = dptr<real>(bhn);
        a.del_v = dptr<real>(bdv);
        if (!run("fct_ale_p1v", st, [&] { return f2a::launch_p1v(plan->dev, a, st); })) return;
        mark_internal(badfh, f2a::p1v_limits_internal(plan->dev, a) ? plan : nullptr, st);
        *alg_state = 7;
        if (!g_resident)
            for (Buffer *b : {bplus, bminus, badfv, bdv})
                if (!d2h_async(b, st)) {
                    *alg_state = 0;
                    return;
                }
        return;
    }
    if (!run("fct_ale_p1", st, [&] { return f2a::launch_p1_fused(plan->dev, a, st); })) return;
    *alg_state = 6;
    if (!g_resident && (!d2h_async(bplus, st) || !d2h_async(bminus, st))) *alg_state = 0;
}

void fct_ale_pre_comm_batched_acc_(int *alg_state, void **s, int *ntracers, void **fct_plus,
                                   void **fct_minus, void **ttf, void **fct_LO, void **fct_adf_v,
                                   void **fct_adf_h, void **area_inv, int *myDim_nod2D,
                                   int *eDim_nod2D, int *myDim_elem2D, int *myDim_edge2D, int *nl,
                                   void **nlevels_nod2D, void **nlevels_elem2D, void **elem2D_nodes,
                                   void **nod_in_elem2D_num, void **nod_in_elem2D,
                                   int *nod_in_elem2D_dim, void **nod2D_edges, void **elem2D_edges,
                                   int *vlimit, real *flux_eps, real *bignumber, real *dt)
{
    pre_comm_fused_impl(alg_state, s, ntracers, fct_plus, fct_minus, ttf, fct_LO, fct_adf_v, fct_adf_h, area_inv,
                        myDim_nod2D, eDim_nod2D, myDim_elem2D, myDim_edge2D, nl, nlevels_nod2D, nlevels_elem2D,
                        elem2D_nodes, nod_in_elem2D_num, nod_in_elem2D, nod_in_elem2D_dim, nod2D_edges,
                        elem2D_edges, vlimit, flux_eps, bignumber, dt, nullptr, nullptr, nullptr, nullptr,
                        "fct_ale_pre_comm_batched_acc_");
}

// Phase 1 + the vertical half of phase 2 (b3v, cv: own columns only, no halo).  Then the exchange
// and fct_ale_post_comm_h_acc_.  Same results as pre_comm + post_comm_c.
void fct_ale_pre_comm_v_acc_(int *alg_state, void **s, int *ntracers, void **fct_plus, void **fct_minus,
                             void **ttf, void **fct_LO, void **fct_adf_v, void **fct_adf_h, void **area_inv,
                             void **area, void **hnode, void **hnode_new, void **del_ttf_advvert,
                             int *myDim_nod2D, int *eDim_nod2D, int *myDim_elem2D, int *myDim_edge2D, int *nl,
                             void **nlevels_nod2D, void **nlevels_elem2D, void **elem2D_nodes,
                             void **nod_in_elem2D_num, void **nod_in_elem2D, int *nod_in_elem2D_dim,
                             void **nod2D_edges, void **elem2D_edges, int *vlimit, real *flux_eps,
                             real *bignumber, real *dt)
{
    if (!area) {
        *alg_state = 0;
        report("fct_ale_pre_comm_v_acc_: area handle missing");
        return;
    }
    pre_comm_fused_impl(alg_state, s, ntracers, fct_plus, fct_minus, ttf, fct_LO, fct_adf_v, fct_adf_h, area_inv,
                        myDim_nod2D, eDim_nod2D, myDim_elem2D, myDim_edge2D, nl, nlevels_nod2D, nlevels_elem2D,
                        elem2D_nodes, nod_in_elem2D_num, nod_in_elem2D, nod_in_elem2D_dim, nod2D_edges,
                        elem2D_edges, vlimit, flux_eps, bignumber, dt, area, hnode, hnode_new, del_ttf_advvert,
                        "fct_ale_pre_comm_v_acc_");
}

// ----------------------------------------------------------------------------- phase 2

void fct_ale_inter_comm_acc_(int *alg_state, void **s, void **fct_plus, void **fct_minus,
                             void **fct_adf_v, int *myDim_nod2D, int *nl, void **nlevels_nod2D)
{
    const PhaseRange range("fct_ale_inter_comm_acc_");
    const hipStream_t st = stream_of(s);
    const int N = *myDim_nod2D, NL = *nl, L = NL - 1;
    if (!check_levels(NL, "fct_ale_inter_comm_acc_")) return;
    Buffer *bplus = need(fct_plus, col_bytes(N, L), "fct_plus"), *bminus = need(fct_minus, col_bytes(N, L), "fct_minus");
    Buffer *badfv = need(fct_adf_v, col_bytes(N, NL), "fct_adf_v");
    Buffer *bnl = need(nlevels_nod2D, sizeof(int) * (size_t)N, "nlevels_nod2D");
    if (!bplus || !bminus || !badfv || !bnl) return;
    if (has_internal(badfv, st)) {
        // fast mode: fct_ale_pre_comm_acc_ limited fct_adf_v already (reference :342-356 computed
        // b3v here); what is left is the reference's transfer back
        mark_internal(badfv, nullptr, st);
        *alg_state = 7;
        if (!g_resident && !d2h_async(badfv, st)) *alg_state = 0;
        return;
    }
    const bool stepwise = kernel_path() == 1;
    if (!run("fct_ale_b3_vertical", st, [&] {
            return stepwise ? f2a::launch_b3v(N, NL, dptr<int>(bnl), dptr<real>(bplus), dptr<real>(bminus), dptr<real>(badfv), st)
                            : f2a::launch_b3v_cols(N, NL, dptr<int>(bnl), dptr<real>(bplus), dptr<real>(bminus),
                                                   dptr<real>(badfv), st);
        }))
        return;
    *alg_state = 7;
    if (!g_resident && !d2h_async(badfv, st)) *alg_state = 0;
}

void fct_ale_post_comm_acc_(int *alg_state, void **s, void **fct_plus, void **fct_minus,
                            void **fct_adf_h, int *myDim_edge2D, int *nl, void **nlevels_elem2D,
                            int *nod_in_elem2D_dim, void **nod2D_edges, void **elem2D_edges)
{
    const PhaseRange range("fct_ale_post_comm_acc_");
    (void)nod_in_elem2D_dim;
    const hipStream_t st = stream_of(s);
    const int E = *myDim_edge2D, NL = *nl, L = NL - 1;
    if (!check_levels(NL, "fct_ale_post_comm_acc_")) return;
    Buffer *bplus = buf(fct_plus, "fct_plus"), *bminus = buf(fct_minus, "fct_minus");
    Buffer *badfh = need(fct_adf_h, col_bytes(E, L), "fct_adf_h");
    Buffer *bnle = buf(nlevels_elem2D, "nlevels_elem2D");
    Buffer *bed = need(nod2D_edges, 2 * sizeof(int) * (size_t)E, "nod2D_edges");
    Buffer *bet = need(elem2D_edges, 2 * sizeof(int) * (size_t)E, "elem2D_edges");
    if (!bplus || !bminus || !badfh || !bnle || !bed || !bet) return;
    // Index validation (every edge node within the plus/minus columns) comes from the edge plan.
    MeshHandles mh;
    mh.edges = bed;
    mh.edge_tri = bet;
    mh.nlev_elem = bnle;
    const int ncols = (int)(std::min(bplus->size, bminus->size) / ((size_t)L * sizeof(real)));
    const Plan *plan = get_plan(mh, 0, ncols, E, NL, false);
    if (!plan) return;
    // fast mode: the block-internal edges were limited by fct_ale_pre_comm_acc_ (marked with its
    // plan, whose lists say which); b3h runs on the others
    const Plan *ip = peek_internal(badfh, st);
    if (has_internal(badfh, st) && !ip) {
        report("fct_ale_post_comm_acc_: the mesh plan that limited part of fct_adf_h was freed");
        return;
    }
    if (ip && (ip->dev.n_edges != E || ip->dev.n_total > ncols)) {
        report("fct_ale_post_comm_acc_: fct_adf_h was partly limited on another mesh");
        return;
    }
    if (!g_resident && (!h2d(bplus, false, st, false) || !h2d(bminus, false, st, false))) return;  // reference :364-365
    // fused path: the production edge kernel over the plan's edge list (edge index order here)
    const bool stepwise = kernel_path() == 1;
    f2a::Tracers tro;
    tro.order = f2a::pass_order(*plan, 1);  // b3h's flux stores (Infinity Cache reuse by the c-step)
    if (!run("fct_ale_b3_horizontal", st, [&] {
            if (ip) {  // interior edges crossing p1v blocks, then the boundary ones
                const f2a::MeshPlanDev &de = ip->dev;
                const hipError_t e = f2a::launch_b3h_ext(de, NL, dptr<real>(bplus), dptr<real>(bminus),
                                                         dptr<real>(badfh), tro, st);
                const int eb = de.n_edge_interior;
                if (e != hipSuccess || eb >= E) return e;
                return f2a::launch_b3h_fused(de, NL, eb, E - eb, dptr<real>(bplus), dptr<real>(bminus),
                                             dptr<real>(badfh), tro, st);
            }
            if (!stepwise && plan->dev.p_edge_info)
                return f2a::launch_b3h_fused(plan->dev, NL, 0, E, dptr<real>(bplus), dptr<real>(bminus), dptr<real>(badfh),
                                             tro, st);
            return f2a::launch_b3h(E, NL, dptr<int>(bnle), dptr<int>(bed), dptr<int>(bet), dptr<real>(bplus),
                                   dptr<real>(bminus), dptr<real>(badfh), st);
        }))
        return;
    mark_internal(badfh, nullptr, st);
    *alg_state = 8;
    if (!g_resident && !d2h_async(badfh, st)) *alg_state = 0;
}

void fct_ale_c_acc_(int *alg_state, void **s, void **del_ttf_advvert, void **del_ttf_advhoriz,
                    void **ttf, void **fct_LO, void **hnode, void **hnode_new, void **fct_adf_v,
                    void **fct_adf_h, void **area, int *myDim_nod2D, int *eDim_nod2D,
                    int *myDim_edge2D, int *nl, void **nlevels_nod2D, void **nlevels_elem2D,
                    void **nod2D_edges, void **elem2D_edges, real *dt)
{
    const PhaseRange range("fct_ale_c_acc_");
    const hipStream_t st = stream_of(s);
    const int N = *myDim_nod2D, NT = N + *eDim_nod2D, E = *myDim_edge2D, NL = *nl, L = NL - 1;
    if (!check_levels(NL, "fct_ale_c_acc_")) return;
    Buffer *bdv = need(del_ttf_advvert, col_bytes(N, L), "del_ttf_advvert");
    Buffer *bdh = need(del_ttf_advhoriz, col_bytes(N, L), "del_ttf_advhoriz");
    Buffer *bttf = need(ttf, col_bytes(N, L), "ttf"), *blo = need(fct_LO, col_bytes(N, L), "fct_LO");
    Buffer *bh = need(hnode, col_bytes(N, L), "hnode"), *bhn = need(hnode_new, col_bytes(N, L), "hnode_new");
    Buffer *badfv = need(fct_adf_v, col_bytes(N, NL), "fct_adf_v"), *badfh = need(fct_adf_h, col_bytes(E, L), "fct_adf_h");
    Buffer *barea = need(area, col_bytes(N, NL), "area");
    Buffer *bnl = need(nlevels_nod2D, sizeof(int) * (size_t)N, "nlevels_nod2D");
    MeshHandles mh;
    mh.edges = need(nod2D_edges, 2 * sizeof(int) * (size_t)E, "nod2D_edges");
    mh.edge_tri = need(elem2D_edges, 2 * sizeof(int) * (size_t)E, "elem2D_edges");
    mh.nlev_elem = buf(nlevels_elem2D, "nlevels_elem2D");
    if (!bdv || !bdh || !bttf || !blo || !bh || !bhn || !badfv || !badfh || !barea || !bnl || !mh.edges || !mh.edge_tri || !mh.nlev_elem)
        return;
    mh.nlev_nod = bnl;
    const Plan *plan = get_plan(mh, N, NT, E, NL, false);
    if (!plan) return;
    const f2a::MeshPlanDev &d = plan->dev;
    if (badfv->cv && badfv->cv->b[0] != bdv) {
        report("fct_ale_c_acc_: del_ttf_advvert is not the one bound to fct_adf_v (fesom2_bind_c_vertical_)");
        return;
    }
    if (has_internal(bdv, st)) {
        // c-vertical was done by pre_comm on the bound fields: they must be this call's, on this mesh
        const CvBinding *cv = badfv->cv;
        if (!cv || cv->b[0] != bdv || cv->b[1] != bh || cv->b[2] != bhn || cv->b[3] != barea) {
            report("fct_ale_c_acc_: del_ttf_advvert holds c-vertical of fields other than this call's "
                   "hnode/hnode_new/area (fesom2_bind_c_vertical_ bound others)");
            return;
        }
        const Plan *vp = peek_internal(bdv, st);
        if (!vp || vp->dev.n_owned != N || vp->dev.nl != NL) {
            report("fct_ale_c_acc_: del_ttf_advvert was updated on another mesh (myDim_nod2D = %d, nl = %d here)", N,
                   NL);
            return;
        }
        // the fast mode's fct_ale_pre_comm_acc_ did c-vertical already: c-horizontal only
        f2a::P2Args a{NL, d.p2_rec, N, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, dptr<real>(barea), nullptr,
                      dptr<real>(badfh), nullptr, dptr<real>(bdh), *dt};
        a.tr.order = f2a::pass_order(*plan, 1);  // kernel directions (Infinity Cache reuse)
        if (!run("fct_ale_p2h", st, [&] { return f2a::launch_p2h(d, a, st); })) return;
        mark_internal(bdv, nullptr, st);
    } else if (kernel_path() != 1 && d.p2_rec && (L % 2 == 0 || L >= 3)) {
        // fused path: cv + ch in one node kernel over the processing order
        f2a::P2Args a{NL, d.p2_rec, N, nullptr, nullptr, dptr<real>(bttf), dptr<real>(blo), dptr<real>(bh),
                      dptr<real>(bhn), dptr<real>(barea), dptr<real>(badfv), dptr<real>(badfh), dptr<real>(bdv),
                      dptr<real>(bdh), *dt};
        if (!run("fct_ale_c", st, [&] { return f2a::launch_c_fused(d, a, st); })) return;
    } else {
        if (!run("fct_ale_c_vertical", st, [&] { return f2a::launch_cv(N, NL, dptr<int>(bnl), dptr<real>(bttf), dptr<real>(bh), dptr<real>(blo), dptr<real>(bhn),
                               dptr<real>(badfv), dptr<real>(barea), dptr<real>(bdv), *dt, st); }))
            return;
        if (!run("fct_ale_c_horizontal", st, [&] { return f2a::launch_ch(plan->dev, NL, dptr<real>(badfh), dptr<real>(barea), dptr<real>(bdh), *dt, st); }))
            return;
    }
    *alg_state = 9;
    if (!g_resident && (!d2h_async(bdv, st) || !d2h_async(bdh, st))) *alg_state = 0;
}

// Fused phase 2 (b3h + b3v + cv + ch).  With comm/halo given, the halo exchange of fct_plus/minus
// runs on the plan's communication stream while b3h and the node kernel process the interior
// (no halo endpoint on any incident edge); the boundary part follows once the halo has arrived.
static void post_comm_c_impl(int *alg_state, void **s, void **fct_plus, void **fct_minus, void **fct_adf_v,
                             void **fct_adf_h, void **del_ttf_advvert, void **del_ttf_advhoriz, void **ttf,
                             void **fct_LO, void **hnode, void **hnode_new, void **area, int *myDim_nod2D,
                             int *eDim_nod2D, int *myDim_edge2D, int *nl, void **nlevels_nod2D,
                             void **nlevels_elem2D, void **nod2D_edges, void **elem2D_edges, real *dt,
                             void **comm, void **halo, int ntr, const char *who)
{
    const PhaseRange range(who);
    const hipStream_t st = stream_of(s);
    const int N = *myDim_nod2D, NT = N + *eDim_nod2D, E = *myDim_edge2D, NL = *nl, L = NL - 1;
    if (!check_levels(NL, who)) return;
    if (ntr < 1) {
        report("%s: ntracers = %d", who, ntr);
        return;
    }
    // one tracer: the reference's sizes; batched: (N+H)-column blocks per tracer (see pre_comm)
    const bool batched = ntr > 1;
    const size_t own = batched ? col_bytes(NT, L) * ntr : col_bytes(N, L);
    Buffer *bplus = need(fct_plus, col_bytes(NT, L) * ntr, "fct_plus"), *bminus = need(fct_minus, col_bytes(NT, L) * ntr, "fct_minus");
    Buffer *bdv = need(del_ttf_advvert, own, "del_ttf_advvert");
    Buffer *bdh = need(del_ttf_advhoriz, own, "del_ttf_advhoriz");
    Buffer *bttf = need(ttf, own, "ttf"), *blo = need(fct_LO, own, "fct_LO");
    Buffer *bh = need(hnode, col_bytes(N, L), "hnode"), *bhn = need(hnode_new, col_bytes(N, L), "hnode_new");
    Buffer *badfv = need(fct_adf_v, batched ? col_bytes(NT, NL) * ntr : col_bytes(N, NL), "fct_adf_v");
    Buffer *badfh = need(fct_adf_h, col_bytes(E, L) * ntr, "fct_adf_h");
    Buffer *barea = need(area, col_bytes(N, NL), "area");
    Buffer *bnl = need(nlevels_nod2D, sizeof(int) * (size_t)N, "nlevels_nod2D");
    MeshHandles mh;
    mh.edges = need(nod2D_edges, 2 * sizeof(int) * (size_t)E, "nod2D_edges");
    mh.edge_tri = need(elem2D_edges, 2 * sizeof(int) * (size_t)E, "elem2D_edges");
    mh.nlev_elem = buf(nlevels_elem2D, "nlevels_elem2D");
    if (!bplus || !bminus || !bdv || !bdh || !bttf || !blo || !bh || !bhn || !badfv || !badfh || !barea || !bnl ||
        !mh.edges || !mh.edge_tri || !mh.nlev_elem)
        return;
    mh.nlev_nod = bnl;
    const Plan *plan = get_plan(mh, N, NT, E, NL, false, ntr > 1);
    if (!plan) return;
    const f2a::MeshPlanDev &d = plan->dev;
    if (has_internal(badfh, st) || has_internal(badfv, st)) {  // part of phase 2 done already
        report("%s: fct_adf_h/fct_adf_v come from fct_ale_pre_comm_v_acc_ (finished by fct_ale_post_comm_h_acc_) or "
               "from the fast mode's fct_ale_pre_comm_acc_ (finished by inter_comm and post_comm)", who);
        return;
    }
    if (!g_resident && !comm && (!h2d(bplus, false, st, false) || !h2d(bminus, false, st, false))) return;
    hipEvent_t halo_done = nullptr;
    if (comm) {
        halo_done = f2a::halo_exchange_async(comm, halo, bplus, bminus, ntr, (size_t)NT * L, st);
        if (!halo_done) return;
    }
    // with an exchange in flight only the interior goes first; otherwise everything at once
    const int e_first = comm ? d.n_edge_interior : E, n_first = comm ? d.n_p2_interior : N;
    f2a::P2Args a{NL, d.p2_rec, n_first, dptr<real>(bplus), dptr<real>(bminus), dptr<real>(bttf), dptr<real>(blo),
                  dptr<real>(bh), dptr<real>(bhn), dptr<real>(barea), dptr<real>(badfv), dptr<real>(badfh),
                  dptr<real>(bdv), dptr<real>(bdh), *dt};
    a.tr = f2a::Tracers{ntr, (size_t)NT * L, (size_t)NT * NL, (size_t)E * L};
    a.tr.order = f2a::pass_order(*plan, ntr);  // kernel directions (Infinity Cache reuse)
    // b3-horizontal as its own edge kernel, then the node kernel (the alternatives measured slower:
    // DESIGN.md §3)
    {
        if (!run("fct_ale_b3_horizontal", st, [&] {
                return f2a::launch_b3h_fused(d, NL, 0, e_first, dptr<real>(bplus), dptr<real>(bminus), dptr<real>(badfh),
                                             a.tr, st);
            }))
            return;
        if (!run("fct_ale_p2", st, [&] { return f2a::launch_p2_fused(d, a, st); })) return;
    }
    if (comm) {
        if (!wait_halo(st, halo_done)) return;
        a.nodes = d.p2_rec + n_first;
        a.count = N - n_first;
        {
            if (!run("fct_ale_b3_horizontal_boundary", st, [&] {
                    return f2a::launch_b3h_fused(d, NL, e_first, E - e_first, dptr<real>(bplus), dptr<real>(bminus),
                                                 dptr<real>(badfh), a.tr, st);
                }))
                return;
            if (!run("fct_ale_p2_boundary", st, [&] { return f2a::launch_p2_fused(d, a, st); })) return;
        }
    }
    *alg_state = 9;
    if (!g_resident)
        for (Buffer *b : {badfv, badfh, bdv, bdh})
            if (!d2h_async(b, st)) {
                *alg_state = 0;
                return;
            }
}

// Horizontal half of phase 2 after fct_ale_pre_comm_v_acc_: [RCCL halo exchange of fct_plus/minus
// overlapped with the interior] + b3h + c-horizontal (comm / halo_plan may be null handles: the
// halo is then already in place).  alg_state -> 9.
void fct_ale_post_comm_h_acc_(int *alg_state, void **s, int *ntracers, void **comm, void **halo_plan,
                              void **fct_plus, void **fct_minus, void **fct_adf_h, void **del_ttf_advhoriz,
                              void **area, int *myDim_nod2D, int *eDim_nod2D, int *myDim_edge2D, int *nl,
                              void **nlevels_nod2D, void **nlevels_elem2D, void **nod2D_edges,
                              void **elem2D_edges, real *dt)
{
    const PhaseRange range("fct_ale_post_comm_h_acc_");
    *alg_state = 0;
    const hipStream_t st = stream_of(s);
    const int N = *myDim_nod2D, NT = N + *eDim_nod2D, E = *myDim_edge2D, NL = *nl, L = NL - 1, ntr = *ntracers;
    if (!check_levels(NL, "fct_ale_post_comm_h_acc_")) return;
    if (ntr < 1) {
        report("fct_ale_post_comm_h_acc_: ntracers = %d", ntr);
        return;
    }
    const bool exch = comm && *comm;
    Buffer *bplus = need(fct_plus, col_bytes(NT, L) * ntr, "fct_plus");
    Buffer *bminus = need(fct_minus, col_bytes(NT, L) * ntr, "fct_minus");
    Buffer *badfh = need(fct_adf_h, col_bytes(E, L) * ntr, "fct_adf_h");
    Buffer *bdh = need(del_ttf_advhoriz, ntr > 1 ? col_bytes(NT, L) * ntr : col_bytes(N, L), "del_ttf_advhoriz");
    Buffer *barea = need(area, col_bytes(N, NL), "area");
    Buffer *bnl = need(nlevels_nod2D, sizeof(int) * (size_t)N, "nlevels_nod2D");
    MeshHandles mh;
    mh.edges = need(nod2D_edges, 2 * sizeof(int) * (size_t)E, "nod2D_edges");
    mh.edge_tri = need(elem2D_edges, 2 * sizeof(int) * (size_t)E, "elem2D_edges");
    mh.nlev_elem = buf(nlevels_elem2D, "nlevels_elem2D");
    if (!bplus || !bminus || !badfh || !bdh || !barea || !bnl || !mh.edges || !mh.edge_tri || !mh.nlev_elem) return;
    mh.nlev_nod = bnl;
    const Plan *plan = get_plan(mh, N, NT, E, NL, false, ntr > 1);
    if (!plan) return;
    const f2a::MeshPlanDev &d = plan->dev;
    // the block-internal edges p1v limited already (fct_ale_pre_comm_v_acc_ marked fct_adf_h with
    // its plan): b3h runs on the other edges of that plan's lists only; the mark is cleared once
    // the whole phase has been enqueued
    const Plan *ip = peek_internal(badfh, st);
    if (has_internal(badfh, st) && !ip) {
        report("fct_ale_post_comm_h_acc_: the mesh plan fct_ale_pre_comm_v_acc_ limited fct_adf_h with was freed");
        return;
    }
    if (!g_resident && !exch && (!h2d(bplus, false, st, false) || !h2d(bminus, false, st, false))) return;
    hipEvent_t halo_done = nullptr;
    if (exch) {
        halo_done = f2a::halo_exchange_async(comm, halo_plan, bplus, bminus, ntr, (size_t)NT * L, st);
        if (!halo_done) return;
    }
    const int e_first = exch ? d.n_edge_interior : E, n_first = exch ? d.n_p2_interior : N;
    f2a::P2Args a{NL, d.p2_rec, n_first, dptr<real>(bplus), dptr<real>(bminus), nullptr, nullptr, nullptr, nullptr,
                  dptr<real>(barea), nullptr, dptr<real>(badfh), nullptr, dptr<real>(bdh), *dt};
    a.tr = f2a::Tracers{ntr, (size_t)NT * L, (size_t)NT * NL, (size_t)E * L};
    a.tr.order = f2a::pass_order(*plan, ntr);  // kernel directions (Infinity Cache reuse)
    const f2a::MeshPlanDev &de = ip ? ip->dev : d;  // the edge lists b3h runs on
    const int eb = de.n_edge_interior;               // boundary edges (a halo endpoint): [eb, E)
    if (!run("fct_ale_b3_horizontal", st, [&] {
            if (ip) {  // interior edges crossing p1v blocks; without an exchange the boundary ones too
                const hipError_t e =
                    f2a::launch_b3h_ext(de, NL, dptr<real>(bplus), dptr<real>(bminus), dptr<real>(badfh), a.tr, st);
                if (e != hipSuccess || exch || eb >= E) return e;
                return f2a::launch_b3h_fused(de, NL, eb, E - eb, dptr<real>(bplus), dptr<real>(bminus),
                                             dptr<real>(badfh), a.tr, st);
            }
            return f2a::launch_b3h_fused(d, NL, 0, e_first, dptr<real>(bplus), dptr<real>(bminus), dptr<real>(badfh),
                                         a.tr, st);
        }))
        return;
    if (!run("fct_ale_p2h", st, [&] { return f2a::launch_p2h(d, a, st); })) return;
    if (exch) {
        if (!wait_halo(st, halo_done)) return;
        if (!run("fct_ale_b3_horizontal_boundary", st, [&] {
                return f2a::launch_b3h_fused(de, NL, eb, E - eb, dptr<real>(bplus), dptr<real>(bminus),
                                             dptr<real>(badfh), a.tr, st);
            }))
            return;
        a.nodes = d.p2_rec + n_first;
        a.count = N - n_first;
        if (!run("fct_ale_p2h_boundary", st, [&] { return f2a::launch_p2h(d, a, st); })) return;
    }
    mark_internal(badfh, nullptr, st);
    *alg_state = 9;
    if (!g_resident && (!d2h_async(badfh, st) || !d2h_async(bdh, st))) *alg_state = 0;
}

void fct_ale_post_comm_c_acc_(int *alg_state, void **s, void **fct_plus, void **fct_minus,
                              void **fct_adf_v, void **fct_adf_h, void **del_ttf_advvert,
                              void **del_ttf_advhoriz, void **ttf, void **fct_LO, void **hnode,
                              void **hnode_new, void **area, int *myDim_nod2D, int *eDim_nod2D,
                              int *myDim_edge2D, int *nl, void **nlevels_nod2D,
                              void **nlevels_elem2D, void **nod2D_edges, void **elem2D_edges,
                              real *dt)
{
    post_comm_c_impl(alg_state, s, fct_plus, fct_minus, fct_adf_v, fct_adf_h, del_ttf_advvert, del_ttf_advhoriz, ttf,
                     fct_LO, hnode, hnode_new, area, myDim_nod2D, eDim_nod2D, myDim_edge2D, nl, nlevels_nod2D,
                     nlevels_elem2D, nod2D_edges, elem2D_edges, dt, nullptr, nullptr, 1, "fct_ale_post_comm_c_acc_");
}

void fct_ale_exchange_post_comm_c_acc_(int *alg_state, void **s, void **comm, void **halo_plan,
                                       void **fct_plus, void **fct_minus, void **fct_adf_v,
                                       void **fct_adf_h, void **del_ttf_advvert, void **del_ttf_advhoriz,
                                       void **ttf, void **fct_LO, void **hnode, void **hnode_new,
                                       void **area, int *myDim_nod2D, int *eDim_nod2D,
                                       int *myDim_edge2D, int *nl, void **nlevels_nod2D,
                                       void **nlevels_elem2D, void **nod2D_edges, void **elem2D_edges,
                                       real *dt)
{
    post_comm_c_impl(alg_state, s, fct_plus, fct_minus, fct_adf_v, fct_adf_h, del_ttf_advvert, del_ttf_advhoriz, ttf,
                     fct_LO, hnode, hnode_new, area, myDim_nod2D, eDim_nod2D, myDim_edge2D, nl, nlevels_nod2D,
                     nlevels_elem2D, nod2D_edges, elem2D_edges, dt, comm, halo_plan, 1,
                     "fct_ale_exchange_post_comm_c_acc_");
}

// Batched fused phase 2 (layouts as fct_ale_pre_comm_batched_acc_; hnode, hnode_new, area shared).
void fct_ale_post_comm_c_batched_acc_(int *alg_state, void **s, int *ntracers, void **fct_plus,
                                      void **fct_minus, void **fct_adf_v, void **fct_adf_h,
                                      void **del_ttf_advvert, void **del_ttf_advhoriz, void **ttf,
                                      void **fct_LO, void **hnode, void **hnode_new, void **area,
                                      int *myDim_nod2D, int *eDim_nod2D, int *myDim_edge2D, int *nl,
                                      void **nlevels_nod2D, void **nlevels_elem2D,
                                      void **nod2D_edges, void **elem2D_edges, real *dt)
{
    post_comm_c_impl(alg_state, s, fct_plus, fct_minus, fct_adf_v, fct_adf_h, del_ttf_advvert, del_ttf_advhoriz, ttf,
                     fct_LO, hnode, hnode_new, area, myDim_nod2D, eDim_nod2D, myDim_edge2D, nl, nlevels_nod2D,
                     nlevels_elem2D, nod2D_edges, elem2D_edges, dt, nullptr, nullptr, *ntracers,
                     "fct_ale_post_comm_c_batched_acc_");
}

// Batched, with the halo exchange of all tracers overlapped with the interior.
void fct_ale_exchange_post_comm_c_batched_acc_(int *alg_state, void **s, void **comm, void **halo_plan,
                                               int *ntracers, void **fct_plus, void **fct_minus,
                                               void **fct_adf_v, void **fct_adf_h, void **del_ttf_advvert,
                                               void **del_ttf_advhoriz, void **ttf, void **fct_LO,
                                               void **hnode, void **hnode_new, void **area,
                                               int *myDim_nod2D, int *eDim_nod2D, int *myDim_edge2D,
                                               int *nl, void **nlevels_nod2D, void **nlevels_elem2D,
                                               void **nod2D_edges, void **elem2D_edges, real *dt)
{
    post_comm_c_impl(alg_state, s, fct_plus, fct_minus, fct_adf_v, fct_adf_h, del_ttf_advvert, del_ttf_advhoriz, ttf,
                     fct_LO, hnode, hnode_new, area, myDim_nod2D, eDim_nod2D, myDim_edge2D, nl, nlevels_nod2D,
                     nlevels_elem2D, nod2D_edges, elem2D_edges, dt, comm, halo_plan, *ntracers,
                     "fct_ale_exchange_post_comm_c_batched_acc_");
}

// iter_yn phase 2 (docs/refactoring.md:227-229, :258-260, :265-290): b3 limiting with the
// remainders (1-ae)*flux into fct_adf_v2/fct_adf_h2, fct_LO updated with the limited fluxes, then
// fct_adf_v <- fct_adf_v2 and fct_adf_h <- fct_adf_h2 (whole arrays, as the Fortran assignment);
// the caller runs the next fct_ale iteration.  alg_state -> 9.
static void post_comm_iter_impl(int *alg_state, void **s, int ntr, void **fct_plus, void **fct_minus,
                                void **fct_adf_v, void **fct_adf_h, void **fct_adf_v2, void **fct_adf_h2,
                                void **fct_LO, void **hnode_new, void **area, int *myDim_nod2D,
                                int *eDim_nod2D, int *myDim_edge2D, int *nl, void **nlevels_nod2D,
                                void **nlevels_elem2D, void **nod2D_edges, void **elem2D_edges, real *dt,
                                const char *who)
{
    const PhaseRange range(who);
    *alg_state = 0;
    const hipStream_t st = stream_of(s);
    const int N = *myDim_nod2D, NT = N + *eDim_nod2D, E = *myDim_edge2D, NL = *nl, L = NL - 1;
    if (!check_levels(NL, who)) return;
    if (ntr < 1) {
        report("%s: ntracers = %d", who, ntr);
        return;
    }
    const bool batched = ntr > 1;
    const size_t node_b = batched ? col_bytes(NT, L) * ntr : col_bytes(N, L);
    const size_t lev_b = batched ? col_bytes(NT, NL) * ntr : col_bytes(N, NL);
    Buffer *bplus = need(fct_plus, col_bytes(NT, L) * ntr, "fct_plus");
    Buffer *bminus = need(fct_minus, col_bytes(NT, L) * ntr, "fct_minus");
    Buffer *badfv = need(fct_adf_v, lev_b, "fct_adf_v"), *badfv2 = need(fct_adf_v2, lev_b, "fct_adf_v2");
    Buffer *badfh = need(fct_adf_h, col_bytes(E, L) * ntr, "fct_adf_h");
    Buffer *badfh2 = need(fct_adf_h2, col_bytes(E, L) * ntr, "fct_adf_h2");
    Buffer *blo = need(fct_LO, node_b, "fct_LO");
    Buffer *bhn = need(hnode_new, col_bytes(N, L), "hnode_new"), *barea = need(area, col_bytes(N, NL), "area");
    Buffer *bnl = need(nlevels_nod2D, sizeof(int) * (size_t)N, "nlevels_nod2D");
    MeshHandles mh;
    mh.edges = need(nod2D_edges, 2 * sizeof(int) * (size_t)E, "nod2D_edges");
    mh.edge_tri = need(elem2D_edges, 2 * sizeof(int) * (size_t)E, "elem2D_edges");
    mh.nlev_elem = buf(nlevels_elem2D, "nlevels_elem2D");
    if (!bplus || !bminus || !badfv || !badfv2 || !badfh || !badfh2 || !blo || !bhn || !barea || !bnl || !mh.edges ||
        !mh.edge_tri || !mh.nlev_elem)
        return;
    mh.nlev_nod = bnl;
    const Plan *plan = get_plan(mh, N, NT, E, NL, false, ntr > 1);
    if (!plan) return;
    const f2a::MeshPlanDev &d = plan->dev;
    if (has_internal(badfh, st) || has_internal(badfv, st)) {  // part of phase 2 done already
        report("%s: fct_adf_h/fct_adf_v come from fct_ale_pre_comm_v_acc_ or the fast mode's fct_ale_pre_comm_acc_; "
               "iter_yn needs the raw fluxes (fesom2_set_path_(0))", who);
        return;
    }
    if (!g_resident) {
        for (Buffer *b : {bplus, bminus, blo, badfv2, badfh2})
            if (!h2d(b, false, st, false)) return;
    }
    const f2a::Tracers trs{ntr, (size_t)NT * L, (size_t)NT * NL, (size_t)E * L};
    f2a::P2IterArgs a{NL, d.p2_rec, N, dptr<int>(mh.edges), dptr<real>(bplus), dptr<real>(bminus), dptr<real>(bhn),
                      dptr<real>(barea), dptr<real>(badfh), dptr<real>(blo), dptr<real>(badfv), dptr<real>(badfv2),
                      *dt, trs};
    if (!run("fct_ale_p2_iter", st, [&] { return f2a::launch_p2_iter(d, a, st); })) return;
    if (!run("fct_ale_b3_horizontal_iter", st, [&] {
            return f2a::launch_b3h_iter(d, NL, dptr<real>(bplus), dptr<real>(bminus), dptr<real>(badfh),
                                        dptr<real>(badfh2), trs, st);
        }))
        return;
    // halo columns of the whole-array fct_adf_v <- fct_adf_v2 (where the handles hold them)
    const size_t need_halo = col_bytes(NT, NL) * ntr;
    if (NT > N && badfv->size >= need_halo && badfv2->size >= need_halo)
        for (int k = 0; k < ntr; k++) {
            const size_t off = (size_t)k * NT * NL + (size_t)N * NL;
            if (!ok(hipMemcpyAsync(dptr<real>(badfv) + off, dptr<real>(badfv2) + off, col_bytes(NT - N, NL),
                                   hipMemcpyDeviceToDevice, st),
                    "hipMemcpyAsync(fct_adf_v halo)"))
                return;
        }
    *alg_state = 9;
    if (!g_resident)
        for (Buffer *b : {blo, badfv, badfv2, badfh, badfh2})
            if (!d2h_async(b, st)) {
                *alg_state = 0;
                return;
            }
}

void fct_ale_post_comm_iter_acc_(int *alg_state, void **s, void **fct_plus, void **fct_minus,
                                 void **fct_adf_v, void **fct_adf_h, void **fct_adf_v2,
                                 void **fct_adf_h2, void **fct_LO, void **hnode_new, void **area,
                                 int *myDim_nod2D, int *eDim_nod2D, int *myDim_edge2D, int *nl,
                                 void **nlevels_nod2D, void **nlevels_elem2D, void **nod2D_edges,
                                 void **elem2D_edges, real *dt)
{
    post_comm_iter_impl(alg_state, s, 1, fct_plus, fct_minus, fct_adf_v, fct_adf_h, fct_adf_v2, fct_adf_h2, fct_LO,
                        hnode_new, area, myDim_nod2D, eDim_nod2D, myDim_edge2D, nl, nlevels_nod2D, nlevels_elem2D,
                        nod2D_edges, elem2D_edges, dt, "fct_ale_post_comm_iter_acc_");
}

void fct_ale_post_comm_iter_batched_acc_(int *alg_state, void **s, int *ntracers, void **fct_plus,
                                         void **fct_minus, void **fct_adf_v, void **fct_adf_h,
                                         void **fct_adf_v2, void **fct_adf_h2, void **fct_LO,
                                         void **hnode_new, void **area, int *myDim_nod2D,
                                         int *eDim_nod2D, int *myDim_edge2D, int *nl,
                                         void **nlevels_nod2D, void **nlevels_elem2D,
                                         void **nod2D_edges, void **elem2D_edges, real *dt)
{
    post_comm_iter_impl(alg_state, s, *ntracers, fct_plus, fct_minus, fct_adf_v, fct_adf_h, fct_adf_v2, fct_adf_h2,
                        fct_LO, hnode_new, area, myDim_nod2D, eDim_nod2D, myDim_edge2D, nl, nlevels_nod2D,
                        nlevels_elem2D, nod2D_edges, elem2D_edges, dt, "fct_ale_post_comm_iter_batched_acc_");
}

// ----------------------------------------------------------------------------- utilities

void fesom2_set_resident_(int *resident) { g_resident = (resident && *resident) ? 1 : 0; }
void fesom2_set_path_(int *path) { set_kernel_path(path ? *path : 0); }

void fesom2_prepare_mesh_(int *istat, int *myDim_nod2D, int *eDim_nod2D, int *myDim_elem2D,
                          int *myDim_edge2D, int *nl, void **nlevels_nod2D, void **nlevels_elem2D,
                          void **elem2D_nodes, void **nod_in_elem2D_num, void **nod_in_elem2D,
                          int *nod_in_elem2D_dim, void **nod2D_edges, void **elem2D_edges)
{
    *istat = 1;
    (void)myDim_elem2D;
    const int N = *myDim_nod2D, NT = N + *eDim_nod2D, E = *myDim_edge2D;
    MeshHandles mh;
    mh.edges = buf(nod2D_edges, "nod2D_edges");
    mh.edge_tri = buf(elem2D_edges, "elem2D_edges");
    mh.nlev_elem = buf(nlevels_elem2D, "nlevels_elem2D");
    Buffer *bnlnod = buf(nlevels_nod2D, "nlevels_nod2D");
    mh.elem_nodes = buf(elem2D_nodes, "elem2D_nodes");
    mh.nie = buf(nod_in_elem2D, "nod_in_elem2D");
    mh.nie_num = buf(nod_in_elem2D_num, "nod_in_elem2D_num");
    mh.dim = *nod_in_elem2D_dim;
    if (!mh.edges || !mh.edge_tri || !mh.nlev_elem || !bnlnod || !mh.elem_nodes || !mh.nie || !mh.nie_num) return;
    mh.nlev_nod = bnlnod;
    // every plan a call on this mesh may ask for: single-tracer and batched (the same object where
    // their shapes resolve alike), with and without the element ring -- so a graph capture of any
    // entry sequence after this call builds nothing
    for (const bool batched : {false, true})
        for (const bool ring : {true, false})
            if (!get_plan(mh, N, NT, E, *nl, ring, batched)) return;
    *istat = 0;
}

// Diagnostics of the mesh plan the phase-1 kernels run on (for the benchmark's byte counts):
// info[0] p1v block columns of the internal-edge lists (0: none), [1] interior edges (both
// endpoints owned), [2] interior edges crossing p1v blocks (b3h's), [3] block-internal edges
// (limited inside p1v), [4] their edge cells (sum of levels); [5, 10) the same for the plan of batched
// calls (ntracers > 1, built here if needed).  *ninfo: entries wanted (<= 10) / written.
// The Infinity-Cache pass order (f2a::pass_order) the split, fused and reference-sequence entries
// use for a call of `ntracers` tracers on this mesh (plan built if needed).
void fesom2_pass_order_(int *istat, int *myDim_nod2D, int *eDim_nod2D, int *myDim_edge2D, int *nl,
                        void **nlevels_nod2D, void **nlevels_elem2D, void **nod2D_edges, void **elem2D_edges,
                        int *ntracers, int *order)
{
    *istat = 1;
    *order = 0;
    const int N = *myDim_nod2D, NT = N + *eDim_nod2D, E = *myDim_edge2D, NL = *nl, ntr = *ntracers;
    if (!check_levels(NL, "fesom2_pass_order_")) return;
    if (ntr < 1) {
        report("fesom2_pass_order_: ntracers = %d", ntr);
        return;
    }
    MeshHandles mh;
    mh.edges = need(nod2D_edges, 2 * sizeof(int) * (size_t)E, "nod2D_edges");
    mh.edge_tri = need(elem2D_edges, 2 * sizeof(int) * (size_t)E, "elem2D_edges");
    mh.nlev_elem = buf(nlevels_elem2D, "nlevels_elem2D");
    mh.nlev_nod = need(nlevels_nod2D, sizeof(int) * (size_t)N, "nlevels_nod2D");
    if (!mh.edges || !mh.edge_tri || !mh.nlev_elem || !mh.nlev_nod) return;
    const Plan *plan = get_plan(mh, N, NT, E, NL, false, ntr > 1);
    if (!plan) return;
    *order = f2a::pass_order(*plan, ntr);
    *istat = 0;
}

void fesom2_mesh_info_(int *istat, int *myDim_nod2D, int *eDim_nod2D, int *myDim_elem2D, int *myDim_edge2D,
                       int *nl, void **nlevels_nod2D, void **nlevels_elem2D, void **elem2D_nodes,
                       void **nod_in_elem2D_num, void **nod_in_elem2D, int *nod_in_elem2D_dim,
                       void **nod2D_edges, void **elem2D_edges, long long *info, int *ninfo)
{
    *istat = 1;
    (void)myDim_elem2D;
    const int N = *myDim_nod2D, NT = N + *eDim_nod2D, E = *myDim_edge2D;
    MeshHandles mh;
    mh.edges = buf(nod2D_edges, "nod2D_edges");
    mh.edge_tri = buf(elem2D_edges, "elem2D_edges");
    mh.nlev_elem = buf(nlevels_elem2D, "nlevels_elem2D");
    mh.nlev_nod = buf(nlevels_nod2D, "nlevels_nod2D");
    mh.elem_nodes = buf(elem2D_nodes, "elem2D_nodes");
    mh.nie = buf(nod_in_elem2D, "nod_in_elem2D");
    mh.nie_num = buf(nod_in_elem2D_num, "nod_in_elem2D_num");
    mh.dim = *nod_in_elem2D_dim;
    if (!mh.edges || !mh.edge_tri || !mh.nlev_elem || !mh.nlev_nod || !mh.elem_nodes || !mh.nie || !mh.nie_num) return;
    const int n = std::min(*ninfo, 14);
    for (int part = 0; part < 2; part++) {  // [0, 5) the single-tracer plan, [5, 10) the batched one
        if (part * 5 >= n) break;
        const Plan *plan = get_plan(mh, N, NT, E, *nl, true, part == 1);
        if (!plan) return;
        const long long v[5] = {plan->dev.int_G, plan->dev.n_edge_interior, plan->dev.n_ext_interior,
                                plan->dev.n_edge_interior - plan->dev.n_ext_interior, plan->int_cells};
        for (int k = 0; k < 5 && part * 5 + k < n; k++) info[part * 5 + k] = v[k];
        // [10, 12) / [12, 14): the plan's cluster unions -- p1v block columns (0 = none), largest union
        const long long u[2] = {plan->dev.cu_G, plan->dev.cu_max};
        for (int k = 0; k < 2 && 10 + 2 * part + k < n; k++) info[10 + 2 * part + k] = u[k];
    }
    *ninfo = n;
    *istat = 0;
}

void fesom2_download_(void **mem, void *host_ptr, int *istat)
{
    Buffer *b = buf(mem, "fesom2_download_");
    *istat = (b && ok(hipMemcpy(host_ptr, b->device_pointer, b->size, hipMemcpyDeviceToHost), "D2H")) ? 0 : 1;
}

void fesom2_upload_(void **mem, void *host_ptr, int *istat)
{
    Buffer *b = buf(mem, "fesom2_upload_");
    if (b) mark_internal(b, nullptr, nullptr);  // new contents
    if (b) b->version++;
    *istat = (b && ok(hipMemcpy(b->device_pointer, host_ptr, b->size, hipMemcpyHostToDevice), "H2D")) ? 0 : 1;
}

void fesom2_free_(void **mem)
{
    Buffer *b = buf(mem, "fesom2_free_");
    if (!b) return;
    drop_plans_of(b);
    untrack_object(b);
    delete b->cv;
    (void)hipFree(b->device_pointer);
    if (b->has_event) (void)hipEventDestroy(b->event);
    b->magic = 0;
    delete b;
    *mem = nullptr;
}

void fesom2_free_stream_(void **stream)
{
    if (!stream || !*stream) return;
    auto *s = static_cast<hipStream_t *>(*stream);
    if (*s) (void)hipStreamDestroy(*s);
    delete s;
    *stream = nullptr;
}

void fesom2_free_pinned_(void **hostptr)
{
    if (hostptr && *hostptr) (void)hipHostFree(*hostptr);
    if (hostptr) *hostptr = nullptr;
}

void fesom2_device_sync_(int *istat) { *istat = ok(hipDeviceSynchronize(), "hipDeviceSynchronize") ? 0 : 1; }

// ---- hipGraph capture of a call sequence (device-resident mode).  Everything the entry points
// enqueue on *s between begin and end -- kernels, the exchange's fork/join onto the halo stream and
// its RCCL send/recv -- becomes one graph; launching it replays the sequence without the host-side
// validation, plan lookups and per-kernel launches.  The meshes' plans must exist already (one
// ordinary pass, or fesom2_prepare_mesh_).  Kernel timing is off on captured streams.
//
// A replay re-runs the captured launches with the arguments read at capture time (buffers, sizes,
// dt/flux_eps/bignumber/vlimit, ntracers, path and FESOM2_* kernel choices) and does not write
// alg_state.  Before each replay it waits on the launch stream for the events of the buffers the
// captured calls would have waited on (transfer_var_async_ uploads, reference :293/:316/:326), and it
// refuses to run if a buffer, halo plan or communicator the capture used has been freed since.
struct GraphHandle {
    static constexpr uint32_t kMagic = 0xF2A6A9F1u;
    uint32_t magic = kMagic;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    CaptureLog log;
};

void fesom2_graph_begin_(int *istat, void **s)
{
    *istat = 1;
    if (!g_resident) {
        report("fesom2_graph_begin_: graph capture needs device-resident mode (fesom2_set_resident_(1))");
        return;
    }
    const hipStream_t st = stream_of(s);
    if (!st) {
        report("fesom2_graph_begin_: the null stream cannot be captured");
        return;
    }
    if (capturing(st)) {
        report("fesom2_graph_begin_: the stream is already being captured");
        return;
    }
    if (!ok(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed), "hipStreamBeginCapture")) return;
    if (!capture_open(st)) {
        report("fesom2_graph_begin_: this thread already has a capture open (end it first)");
        hipGraph_t g = nullptr;
        if (hipStreamEndCapture(st, &g) == hipSuccess && g) (void)hipGraphDestroy(g);
        return;
    }
    *istat = 0;
}

void fesom2_graph_end_(int *istat, void **s, void **graph)
{
    *istat = 1;
    *graph = nullptr;
    const hipStream_t st = stream_of(s);
    auto *g = new GraphHandle;
    bool foreign = false;
    if (!capture_close(st, &g->log, &foreign)) {
        if (foreign) {
            // opened on another thread: end the HIP capture and drop the graph, so that no capture
            // stays open (an open capture blocks every plan build in the process)
            report("fesom2_graph_end_: the capture was opened on another thread; it is ended and dropped");
            hipGraph_t dropped = nullptr;
            if (hipStreamEndCapture(st, &dropped) == hipSuccess && dropped) (void)hipGraphDestroy(dropped);
        } else {
            report("fesom2_graph_end_: the stream has no capture opened by fesom2_graph_begin_");
        }
        delete g;
        return;
    }
    if (!ok(hipStreamEndCapture(st, &g->graph), "hipStreamEndCapture") ||
        !ok(hipGraphInstantiate(&g->exec, g->graph, nullptr, nullptr, 0), "hipGraphInstantiate")) {
        if (g->graph) (void)hipGraphDestroy(g->graph);
        delete g;
        return;
    }
    *graph = g;
    *istat = 0;
}

void fesom2_graph_launch_(int *istat, void **graph, void **s)
{
    *istat = 1;
    auto *g = graph && *graph ? static_cast<GraphHandle *>(*graph) : nullptr;
    if (!g || g->magic != GraphHandle::kMagic) {
        report("fesom2_graph_launch_: invalid graph handle");
        return;
    }
    for (const CapturedUse &u : g->log.uses)
        if (!object_live(u.p, u.serial)) {
            report("fesom2_graph_launch_: a buffer, halo plan or communicator the graph captured has been "
                   "freed since the capture (capture again)");
            return;
        }
    if (!marks_replayable(g->log)) return;
    const hipStream_t st = stream_of(s);
    for (const CapturedUse &w : g->log.waits) {
        const Buffer *b = static_cast<const Buffer *>(w.p);
        if (!ok(hipStreamWaitEvent(st, b->event, 0), "hipStreamWaitEvent(graph launch)")) return;
    }
    if (!ok(hipGraphLaunch(g->exec, st), "hipGraphLaunch")) return;
    marks_apply(g->log);  // the host state the captured calls left behind (fct_adf_h's mark)
    *istat = 0;
}

// objects a graph used / buffer events it waits on before each replay (tests and diagnostics)
void fesom2_graph_info_(void **graph, int *n_uses, int *n_waits)
{
    auto *g = graph && *graph ? static_cast<GraphHandle *>(*graph) : nullptr;
    const bool valid = g && g->magic == GraphHandle::kMagic;
    *n_uses = valid ? (int)g->log.uses.size() : -1;
    *n_waits = valid ? (int)g->log.waits.size() : -1;
}

void fesom2_graph_free_(void **graph)
{
    auto *g = graph && *graph ? static_cast<GraphHandle *>(*graph) : nullptr;
    if (!g || g->magic != GraphHandle::kMagic) return;
    (void)hipGraphExecDestroy(g->exec);
    (void)hipGraphDestroy(g->graph);
    g->magic = 0;
    delete g;
    *graph = nullptr;
}

const char *fesom2_last_error(void) { return last_error(); }

void fesom2_event_create_(void **ev, int *istat)
{
    auto *e = new hipEvent_t;
    *istat = ok(hipEventCreate(e), "hipEventCreate") ? 0 : 1;
    *ev = e;
}

void fesom2_event_record_(void **ev, void **s) { (void)hipEventRecord(*static_cast<hipEvent_t *>(*ev), stream_of(s)); }

void fesom2_event_elapsed_(void **ev0, void **ev1, float *ms)
{
    hipEvent_t e0 = *static_cast<hipEvent_t *>(*ev0), e1 = *static_cast<hipEvent_t *>(*ev1);
    (void)hipEventSynchronize(e1);
    if (!ok(hipEventElapsedTime(ms, e0, e1), "hipEventElapsedTime")) *ms = -1.f;
}

void fesom2_event_free_(void **ev)
{
    if (!ev || !*ev) return;
    auto *e = static_cast<hipEvent_t *>(*ev);
    (void)hipEventDestroy(*e);
    delete e;
    *ev = nullptr;
}

}  // extern "C"
