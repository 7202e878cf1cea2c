// halo_rccl.hip -- device-resident halo exchange of fct_plus / fct_minus over RCCL (xGMI).
//
// The reference leaves `call exchange_nod(fct_plus, fct_minus)` (docs/refactoring.md:199-200,
// :235) to the Fortran host: D2H of both arrays (src/fesom2-accelerate.cu:338-339), host MPI, and
// H2D again (:364-365).  Here the exchange stays on the GPU: the owned columns a neighbour needs are
// packed into one contiguous buffer, sent with grouped ncclSend/ncclRecv (point-to-point, which is
// what xGMI links are: no ring collective), and unpacked into the halo columns, all enqueued on the
// caller's stream.  One communicator per process/GPU (one rank per GPU).
#include "f2a_host.hpp"

#include <rccl/rccl.h>

#include <cstring>
#include <vector>

using namespace f2a;

namespace {

struct Comm {
    static constexpr uint32_t kMagic = 0xF2AC0111u;
    uint32_t magic = kMagic;
    ncclComm_t comm = nullptr;
    int rank = 0, nranks = 1;
    uint64_t serial = 0;  // track_object
};

struct HaloPlan {
    static constexpr uint32_t kMagic = 0xF2A4A105u;
    uint32_t magic = kMagic;
    uint64_t serial = 0;  // track_object
    int L = 0;
    std::vector<int> ranks, scount, rcount, soff, roff;  // offsets in columns
    int nsend = 0, nrecv = 0, max_col = -1;
    int *d_send = nullptr, *d_recv = nullptr;  // 0-based local columns
    real *sbuf = nullptr, *rbuf = nullptr;     // [list position][tracer][plus L | minus L]
    int buf_tracers = 0;                       // tracers the buffers hold
    DeviceArrays mem;
    // communication stream + events of the overlapped exchange (created on first use)
    hipStream_t cstream = nullptr;
    hipEvent_t ev_ready = nullptr, ev_done = nullptr;
    ~HaloPlan()
    {
        if (cstream) (void)hipStreamDestroy(cstream);
        if (ev_ready) (void)hipEventDestroy(ev_ready);
        if (ev_done) (void)hipEventDestroy(ev_done);
    }
};

bool nccl_ok(ncclResult_t r, const char *what)
{
    if (r == ncclSuccess) return true;
    report("RCCL error in %s: %s", what, ncclGetErrorString(r));
    return false;
}

Comm *comm_of(void **h)
{
    if (!h || !*h || static_cast<Comm *>(*h)->magic != Comm::kMagic) {
        report("invalid communicator handle");
        return nullptr;
    }
    Comm *c = static_cast<Comm *>(*h);
    note_use(c, c->serial);
    return c;
}

HaloPlan *plan_of(void **h)
{
    if (!h || !*h || static_cast<HaloPlan *>(*h)->magic != HaloPlan::kMagic) {
        report("invalid halo plan handle");
        return nullptr;
    }
    HaloPlan *p = static_cast<HaloPlan *>(*h);
    note_use(p, p->serial);
    return p;
}

// pack/recv buffers for ntr tracers (grown on first use by a larger batch; the old ones stay in
// the plan's arena until it is freed)
bool reserve_tracers(HaloPlan *p, int ntr)
{
    if (ntr <= p->buf_tracers) return true;
    const size_t w = sizeof(real) * 2 * (size_t)p->L * ntr;
    p->sbuf = static_cast<real *>(p->mem.alloc(w * std::max(p->nsend, 1)));
    p->rbuf = static_cast<real *>(p->mem.alloc(w * std::max(p->nrecv, 1)));
    if (!p->sbuf || !p->rbuf) return false;
    p->buf_tracers = ntr;
    return true;
}

}  // namespace

extern "C" {

void fesom2_comm_unique_id_(char *id128, int *istat)
{
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    ncclUniqueId id;
    *istat = nccl_ok(ncclGetUniqueId(&id), "ncclGetUniqueId") ? 0 : 1;
    memcpy(id128, &id, sizeof id);
}

void fesom2_comm_init_(void **comm, char *id128, int *rank, int *nranks, int *istat)
{
    *istat = 1;
    auto *c = new Comm;
    ncclUniqueId id;
    memcpy(&id, id128, sizeof id);
    c->rank = *rank;
    c->nranks = *nranks;
    if (!nccl_ok(ncclCommInitRank(&c->comm, *nranks, id, *rank), "ncclCommInitRank")) {
        delete c;
        *comm = nullptr;
        return;
    }
    c->serial = track_object(c);
    *comm = c;
    *istat = 0;
}

void fesom2_comm_free_(void **comm)
{
    Comm *c = comm_of(comm);
    if (!c) return;
    untrack_object(c);
    (void)ncclCommDestroy(c->comm);
    c->magic = 0;
    delete c;
    *comm = nullptr;
}

void fesom2_comm_info_(void **comm, int *rank, int *nranks, int *device, int *istat)
{
    *istat = 1;
    Comm *c = comm_of(comm);
    if (!c) return;
    if (!nccl_ok(ncclCommUserRank(c->comm, rank), "ncclCommUserRank") ||
        !nccl_ok(ncclCommCount(c->comm, nranks), "ncclCommCount") ||
        !nccl_ok(ncclCommCuDevice(c->comm, device), "ncclCommCuDevice"))
        return;
    *istat = 0;
}

void fesom2_halo_plan_(void **plan, int *nneigh, int *neigh_ranks, int *send_counts,
                       int *send_nodes, int *recv_counts, int *recv_nodes, int *nl, int *istat)
{
    *istat = 1;
    *plan = nullptr;
    if (*nl < 2 || *nneigh < 0) {
        report("fesom2_halo_plan_: nl = %d, nneigh = %d", *nl, *nneigh);
        return;
    }
    auto p = new HaloPlan;
    p->L = *nl - 1;
    std::vector<int> snodes, rnodes;
    for (int k = 0; k < *nneigh; k++) {
        if (send_counts[k] < 0 || recv_counts[k] < 0) {
            report("fesom2_halo_plan_: negative count for neighbour %d", k);
            delete p;
            return;
        }
        p->ranks.push_back(neigh_ranks[k]);
        p->scount.push_back(send_counts[k]);
        p->rcount.push_back(recv_counts[k]);
        p->soff.push_back(p->nsend);
        p->roff.push_back(p->nrecv);
        p->nsend += send_counts[k];
        p->nrecv += recv_counts[k];
    }
    for (int i = 0; i < p->nsend + p->nrecv; i++) {
        const int v = (i < p->nsend ? send_nodes[i] : recv_nodes[i - p->nsend]) - 1;
        if (v < 0) {
            report("fesom2_halo_plan_: node number %d < 1", v + 1);
            delete p;
            return;
        }
        (i < p->nsend ? snodes : rnodes).push_back(v);
        p->max_col = std::max(p->max_col, v);
    }
    p->d_send = p->mem.upload(snodes);
    p->d_recv = p->mem.upload(rnodes);
    if (!p->d_send || !p->d_recv || !reserve_tracers(p, 1)) {
        delete p;
        return;
    }
    p->serial = track_object(p);
    *plan = p;
    *istat = 0;
}

void fesom2_halo_plan_free_(void **plan)
{
    HaloPlan *p = plan_of(plan);
    if (!p) return;
    untrack_object(p);
    p->magic = 0;
    delete p;
    *plan = nullptr;
}

}  // extern "C"

// pack -> grouped send/recv -> unpack, all on stream st (ntr tracers, `stride` doubles apart)
// (bm may be null: one field)
static bool exchange_on(Comm *c, HaloPlan *p, Buffer *bp, Buffer *bm, int ntr, size_t stride, hipStream_t st)
{
    if (!reserve_tracers(p, ntr)) return false;
    real *pa = dptr<real>(bp), *pb = bm ? dptr<real>(bm) : nullptr;
    const size_t w = (bm ? 2 : 1) * (size_t)p->L * ntr;  // doubles per list position
    if (!ok(launch_halo_pack(p->d_send, p->nsend, p->L, ntr, stride, pa, pb, p->sbuf, st), "halo pack"))
        return false;
    if (!nccl_ok(ncclGroupStart(), "ncclGroupStart")) return false;
    for (size_t k = 0; k < p->ranks.size(); k++) {
        if (p->scount[k] &&
            !nccl_ok(ncclSend(p->sbuf + p->soff[k] * w, p->scount[k] * w, ncclDouble, p->ranks[k], c->comm, st), "ncclSend")) {
            (void)ncclGroupEnd();
            return false;
        }
        if (p->rcount[k] &&
            !nccl_ok(ncclRecv(p->rbuf + p->roff[k] * w, p->rcount[k] * w, ncclDouble, p->ranks[k], c->comm, st), "ncclRecv")) {
            (void)ncclGroupEnd();
            return false;
        }
    }
    if (!nccl_ok(ncclGroupEnd(), "ncclGroupEnd")) return false;
    return ok(launch_halo_unpack(p->d_recv, p->nrecv, p->L, ntr, stride, p->rbuf, pa, pb, st), "halo unpack");
}

static bool check_buffers(HaloPlan *p, Buffer *bp, Buffer *bm, int ntr, size_t stride)
{
    if (ntr < 1 || (ntr > 1 && stride < (size_t)(p->max_col + 1) * p->L)) {
        report("halo exchange: %d tracers %zu doubles apart do not fit columns up to %d", ntr, stride, p->max_col + 1);
        return false;
    }
    const size_t need_bytes = sizeof(real) * (stride * (ntr - 1)) + col_bytes(p->max_col + 1, p->L);
    for (Buffer *b : {bp, bm})
        if (b && b->size < need_bytes) {
            report("a field of the exchange holds %zu bytes, the halo plan needs %zu", b->size, need_bytes);
            return false;
        }
    return true;
}

namespace f2a {
hipEvent_t halo_exchange_async(void **comm, void **plan, Buffer *bp, Buffer *bm, int ntr, size_t stride, hipStream_t s)
{
    const PhaseRange range("halo_exchange_async");
    Comm *c = comm_of(comm);
    HaloPlan *p = plan_of(plan);
    if (!c || !p || !check_buffers(p, bp, bm, ntr, stride)) return nullptr;
    if (!p->cstream) {
        if (!ok(hipStreamCreateWithFlags(&p->cstream, hipStreamNonBlocking), "hipStreamCreate(halo)") ||
            !ok(hipEventCreateWithFlags(&p->ev_ready, hipEventDisableTiming), "hipEventCreate(halo)") ||
            !ok(hipEventCreateWithFlags(&p->ev_done, hipEventDisableTiming), "hipEventCreate(halo)"))
            return nullptr;
    }
    if (!ok(hipEventRecord(p->ev_ready, s), "hipEventRecord(halo ready)") ||
        !ok(hipStreamWaitEvent(p->cstream, p->ev_ready, 0), "hipStreamWaitEvent(halo ready)"))
        return nullptr;
    // timed as "halo_exchange" (pack, grouped send/recv, unpack on the halo stream) when timing is on
    void *tok = nullptr;
    if (timing_enabled("halo_exchange") && !capturing(s)) timing_begin("halo_exchange", p->cstream, &tok);
    const bool sent = exchange_on(c, p, bp, bm, ntr, stride, p->cstream);
    if (tok) timing_end(tok, p->cstream);
    if (!sent) return nullptr;
    if (!ok(hipEventRecord(p->ev_done, p->cstream), "hipEventRecord(halo done)")) return nullptr;
    return p->ev_done;
}
}  // namespace f2a

extern "C" {

void fct_ale_exchange_acc_(int *istat, void **s, void **comm, void **plan, void **fct_plus,
                           void **fct_minus)
{
    const PhaseRange range("fct_ale_exchange_acc_");
    *istat = 1;
    Comm *c = comm_of(comm);
    HaloPlan *p = plan_of(plan);
    Buffer *bp = buf(fct_plus, "fct_plus"), *bm = buf(fct_minus, "fct_minus");
    if (!c || !p || !bp || !bm || !check_buffers(p, bp, bm, 1, 0)) return;
    if (exchange_on(c, p, bp, bm, 1, 0, stream_of(s))) *istat = 0;
}

void fct_ale_exchange_batched_acc_(int *istat, void **s, void **comm, void **plan, int *ntracers,
                                   int *nod_columns, void **fct_plus, void **fct_minus)
{
    const PhaseRange range("fct_ale_exchange_batched_acc_");
    *istat = 1;
    Comm *c = comm_of(comm);
    HaloPlan *p = plan_of(plan);
    Buffer *bp = buf(fct_plus, "fct_plus"), *bm = buf(fct_minus, "fct_minus");
    if (!c || !p || !bp || !bm) return;
    const size_t stride = (size_t)(*nod_columns) * p->L;
    if (!check_buffers(p, bp, bm, *ntracers, stride)) return;
    if (exchange_on(c, p, bp, bm, *ntracers, stride, stream_of(s))) *istat = 0;
}

// FESOM's exchange_nod(a) / exchange_nod(a, b) for (nl-1, nod) fields on the device: ttf/fct_LO
// before phase 1, del_ttf_* after the c-step, fct_LO between iter_yn iterations.
// field_b may be a null handle (one field); ntracers blocks nod_columns*(nl-1) doubles apart.
void fesom2_exchange_nod_acc_(int *istat, void **s, void **comm, void **plan, int *ntracers,
                             int *nod_columns, void **field_a, void **field_b)
{
    const PhaseRange range("fesom2_exchange_nod_acc_");
    *istat = 1;
    Comm *c = comm_of(comm);
    HaloPlan *p = plan_of(plan);
    Buffer *ba = buf(field_a, "field_a");
    Buffer *bb = (field_b && *field_b) ? buf(field_b, "field_b") : nullptr;
    if (!c || !p || !ba || (field_b && *field_b && !bb)) return;
    const size_t stride = (size_t)(*nod_columns) * p->L;
    if (!check_buffers(p, ba, bb, *ntracers, stride)) return;
    if (exchange_on(c, p, ba, bb, *ntracers, stride, stream_of(s))) *istat = 0;
}

}  // extern "C"
