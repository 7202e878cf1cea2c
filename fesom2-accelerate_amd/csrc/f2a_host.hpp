// f2a_host.hpp -- host-side helpers shared by the C-ABI translation units.
#pragma once
#include "f2a_internal.hpp"

#include <rocprofiler-sdk-roctx/roctx.h>
#include "../../include/fesom2-accelerate.h"

#include <memory>
#include <string>
#include <vector>

namespace f2a {

// roctx range over one ABI entry (rocprofv3 --marker-trace shows the phases; no-op otherwise)
struct PhaseRange {
    explicit PhaseRange(const char *name) { roctxRangePush(name); }
    ~PhaseRange() { roctxRangePop(); }
    PhaseRange(const PhaseRange &) = delete;
    PhaseRange &operator=(const PhaseRange &) = delete;
};


// ---- error reporting (stderr + thread-local last error, like the reference's errorHandling,
//      include/fesom2-accelerate.h:38-46)
void report(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
bool ok(hipError_t st, const char *what);
const char *last_error();
unsigned long error_count();  // number of report() calls so far (all threads)

// ---- global modes
extern int g_resident;  // fesom2_set_resident_
int kernel_path();      // 0 fused, 1 stepwise, 2 reference-sequence fast mode (fesom2_set_path_;
                        // FESOM2_PATH, read once, sets the default)
void set_kernel_path(int p);

// ---- handles
Buffer *buf(void **h, const char *name);
Buffer *need(void **h, size_t bytes, const char *name);
hipStream_t stream_of(void **s);
Buffer *allocate(void *host, size_t bytes, bool create_event);
bool h2d(Buffer *b, bool sync, hipStream_t s, bool record);
bool d2h_async(Buffer *b, hipStream_t s);
void wait_event(Buffer *b, hipStream_t s);
template <class T>
inline T *dptr(Buffer *b)
{
    return static_cast<T *>(b->device_pointer);
}
inline size_t col_bytes(long cols, int stride) { return (size_t)cols * stride * sizeof(real); }
bool check_levels(int nl, const char *who);

// ---- live objects (Buffer, halo plan, communicator): a serial per live object, so a graph replay
//      can refuse to run when something it captured has been freed (or freed and reallocated at
//      the same address) since the capture.
uint64_t track_object(const void *p);  // register p, return its fresh serial
void untrack_object(const void *p);
bool object_live(const void *p, uint64_t serial);
// Called by every handle lookup: while this thread has a capture open (fesom2_graph_begin_), p is
// recorded as used by the graph.  (Eager calls of the same thread on other streams are recorded
// too; that only makes the replay's liveness check stricter.)
void note_use(const void *p, uint64_t serial);

// ---- hipGraph capture (fesom2_graph_begin_ / _end_ / _launch_).  Decided per stream: a stream is
//      captured if it is the origin of an open capture or was forked into one (the halo stream).
bool capturing(hipStream_t s);
// some capture opened by fesom2_graph_begin_ is still open (any stream, any thread): plan builds
// copy with hipMemcpy, which synchronises the blocking streams and would break it
bool any_capture();
// What a capture recorded: the objects its calls used, and the buffers whose events (recorded by
// transfer_var_async_ outside the capture, which a captured stream may not wait on) every replay
// must wait for before it starts.
struct CapturedUse {
    const void *p;
    uint64_t serial;
};
// fct_adf_h's internal-edge mark (Buffer::int_plan) as a capture saw it.  The mark is host state,
// so a replay has to reproduce it: the captured calls' last write is applied after every launch,
// and when the capture's first access was a read (a captured post_comm_h after an eager
// pre_comm_v), every launch first checks that the mark holds what the capture read.  At capture end
// the mark is put back to its value before the capture: capturing is not running.
struct CapturedMark {
    Buffer *b;
    uint64_t serial;                 // b's live-object serial
    const void *entry;               // the mark before the capture touched it
    uint64_t entry_serial;
    bool read_first = false;         // the capture's first access read the mark
    bool written = false;            // the capture wrote it; final = the last value written
    const void *final_mark = nullptr;
    uint64_t final_serial = 0;
};
struct CaptureLog {
    std::vector<CapturedUse> uses, waits;
    std::vector<CapturedMark> marks;
};
// register an open capture whose origin is s (after hipStreamBeginCapture); false if this thread
// already has one open
bool capture_open(hipStream_t s);
// unregister the capture whose origin is s and hand over its log; false if s is not the origin of
// a capture opened by capture_open on this thread.  A capture whose origin is s but which another
// thread opened is unregistered as well (*foreign = true, return false): the caller ends the HIP
// capture and drops the graph, and that thread's next library call forgets it.
bool capture_close(hipStream_t s, CaptureLog *log, bool *foreign);
// before every replay: the marks whose first captured access was a read must hold what the capture
// read (false + report otherwise); after it: the captured final marks
bool marks_replayable(const CaptureLog &log);
void marks_apply(const CaptureLog &log);
// the captured call on stream s would wait for b's event: record the wait in the log of the
// capture s belongs to (false if s is not in a capture opened by capture_open)
bool defer_event_wait(Buffer *b, hipStream_t s);

// ---- per-kernel timing (fesom2_kernel_timing_): HIP events recorded around each launch on the
//      launch stream while enabled; resolved when the statistics are read.
bool timing_enabled(const char *name);
void timing_begin(const char *name, hipStream_t s, void **token);
void timing_end(void *token, hipStream_t s);
// Launch through `f` with optional timing; reports failures under `name`.
template <class F>
bool run(const char *name, hipStream_t s, F &&f)
{
    void *tok = nullptr;
    if (timing_enabled(name) && !capturing(s)) timing_begin(name, s, &tok);
    const bool good = ok(f(), name);
    if (tok) timing_end(tok, s);
    return good;
}

// The caller's stream waits for the overlapped halo exchange (event `done`).  With timing on, the
// wait itself is timed as "halo_wait": from the stream reaching it (its interior work done) to the
// exchange's completion, i.e. the part of the exchange the interior work did not hide.
inline bool wait_halo(hipStream_t st, hipEvent_t done)
{
    void *tok = nullptr;
    if (timing_enabled("halo_wait") && !capturing(st)) timing_begin("halo_wait", st, &tok);
    const bool good = ok(hipStreamWaitEvent(st, done, 0), "hipStreamWaitEvent(halo)");
    if (tok) timing_end(tok, st);
    return good;
}

// ---- device allocations owned by a plan (freed with it)
struct DeviceArrays {
    std::vector<void *> ptrs;
    ~DeviceArrays();
    void *alloc(size_t bytes);
    template <class T>
    T *upload(const std::vector<T> &v)
    {
        T *p = static_cast<T *>(alloc(v.size() * sizeof(T)));
        if (p && !v.empty() && !ok(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice), "H2D(plan)"))
            return nullptr;
        return p;
    }
};

// ---- derived mesh structures
struct HostMesh {  // host views of the connectivity a plan is built from (nullptr = absent)
    const int *edges = nullptr, *edge_tri = nullptr, *nlev_elem = nullptr, *nlev_nod = nullptr;
    const int *elem_nodes = nullptr, *nie = nullptr, *nie_num = nullptr;
    long n_elem_total = 0;
    int dim = 0;
};

struct ResolvedShape {
    int patch = 0;          // nodes per BFS patch, 0: by numbering (16384 / 4096), 1: index order
    int gshift = 0;         // MeshPlanDev::gshift
    int gcols = 0;          // MeshPlanDev::gcols (0: natural column count << gshift)
    bool large = false;     // row pairs + LDS stash (automatic shape on a large partition)
    bool internal = false;  // block-internal edges limited in p1v (FESOM2_P1V_B3H forces it)
    int strip = 0;          // strip width inside a patch (strip_order), 0: none
    int union_cap = 0;      // > 0: cluster unions of at most this many columns per p1v block, in row pairs
    bool operator==(const ResolvedShape &o) const
    {
        return patch == o.patch && gshift == o.gshift && gcols == o.gcols && large == o.large &&
               internal == o.internal && strip == o.strip && union_cap == o.union_cap;
    }
};

struct Plan {
    MeshPlanDev dev;
    DeviceArrays mem;
    uint64_t serial = 0;  // track_object (fct_adf_h's internal-edge marker refers to a plan)
    long long int_cells = 0;  // edge cells of the block-internal edges p1v limits
    int num_kernels = 10;     // stepwise phase 1 stops after this many reference steps
    int cache_order = -1;     // plan option FESOM2_CACHE_ORDER: -1 automatic, 0 off, 1 on (pass_order)
    bool has_ring = false;
    int lmax_edges = 0;
    // what the plan was built for: its resolved shape (under the plan options read at build time)
    // and the owned wet cells the size rules saw -- a batched call shares a single-tracer plan only
    // when its own shape resolves to the same (get_plan)
    ResolvedShape shape;
    long long wet_cells = 0;
};

// Tracers::order of a direction-split or fused pass of `ntr` tracers on `plan`.  When the pass's
// fct_adf_h fits the 256 MiB Infinity Cache with room to spare (ntr * edges * (nl-1) * 8 B <=
// kCacheOrderBytes, e.g. 127k x 47: 143 MB), the kernels alternate directions -- phase 1 walks each
// XCD's tile range backwards, b3h forwards, the node kernel of phase 2 backwards -- so each kernel
// starts on the lines its predecessor touched last, and b3h stores the limited fluxes
// cache-allocating for the node kernel; the next pass's phase 1 starts where this pass's phase 2
// began, i.e. on the cold end (no gain from repeating a benchmark's inputs).  Larger passes keep
// every kernel forwards with non-temporal flux stores (measured).
constexpr long long kCacheOrderBytes = 192ll << 20;
int pass_order(const Plan &plan, int ntr);

// Processing-order options of a plan.  Single-tracer calls use the defaults (16384-node patches
// for a numbering with locality, the natural block size); calls with ntracers > 1 get a plan of
// their own (get_plan(..., batched)): on large partitions 4096-node patches and smaller blocks, because a batch's
// tiles run (column group, tracer) tracer-fastest, which puts a column's reuse by the next row of
// the patch ntracers times more tiles later -- beyond the XCD L2's lifetime with wide patches
// (batched plan).
struct PlanShape {
    static constexpr int kAuto = 99;
    int patch = 0;   // nodes per BFS patch; 0: automatic (16384 / 4096 by numbering); 1: index order;
                     // kAuto (batched): 4096 where the blocks are smaller, else automatic
    int gshift = 0;  // MeshPlanDev::gshift; kAuto (batched): on partitions of >= 32M wet cells the
                     // largest column count below the natural one with >= 90 % of the lanes busy
    int gcols = 0;   // MeshPlanDev::gcols: columns per block (> 0 overrides gshift)
    int strip = 0;   // nodes per strip row inside a patch (strip_order; 0: none); kAuto (batched): by size
};
// the shape of the single-tracer (batched = false) or the batched plan, with the plan options
// FESOM2_PATCH / FESOM2_BATCH_PATCH and FESOM2_BATCH_GROUP_SHIFT (read when the plan is built)
PlanShape plan_shape(bool batched);

// A shape with the automatic rules applied for a partition of `wet_cells` owned wet cells.  The
// large-partition rules (smaller blocks in row pairs, the internal edges' LDS stash, the
// block-internal edges limited in p1v) start at large_partition_cells() = 32M wet cells; the plan
// option FESOM2_LARGE_CELLS moves that threshold (tests run the large plan on small meshes with
// it).  Two shapes that resolve alike give the same plan: get_plan then shares one plan between
// single-tracer and batched calls (every partition below the threshold).
long long large_partition_cells();
ResolvedShape resolve_shape(const PlanShape &s, long long wet_cells, int nl);

// Node->edge CSR for nodes [0, n_csr) in ascending edge order; clusters for [0, n_owned) when the
// element connectivity is present.  Validates every index; returns nullptr with `err` set.
std::unique_ptr<Plan> build_plan(const HostMesh &m, int n_owned, int n_total, int n_edges,
                                 int n_csr, int nl, const PlanShape &shape, std::string &err);

struct MeshHandles {
    Buffer *edges = nullptr, *edge_tri = nullptr, *nlev_elem = nullptr, *nlev_nod = nullptr;
    Buffer *elem_nodes = nullptr, *nie = nullptr, *nie_num = nullptr;
    int dim = 0;
};
// Cached per (handles, partition sizes, batched); built synchronously on first use.  `batched`: the
// plan of calls with ntracers > 1 (PlanShape) -- the single-tracer plan itself (one object under
// both keys) when the two shapes resolve alike (ResolvedShape).
const Plan *get_plan(const MeshHandles &h, int n_owned, int n_total, int n_edges, int nl,
                     bool with_ring, bool batched = false);
void drop_plans_of(const Buffer *b);
// Phase marks (Buffer::int_plan) -- part of phase 2 already done by a phase-1 launch: on fct_adf_h
// the block-internal edges of `plan` limited by p1v (fct_ale_pre_comm_v_acc_, or fct_ale_pre_comm_acc_
// in the fast mode); on fct_adf_v b3-vertical done by fct_ale_pre_comm_acc_ in the fast mode
// (fct_ale_inter_comm_acc_ then has nothing left to compute).  nullptr clears.  `s` is the stream of the call (nullptr for the
// synchronous uploads): on a captured stream the access is recorded in the capture's log.
void mark_internal(Buffer *adf_h, const Plan *plan, hipStream_t s);
bool has_internal(Buffer *adf_h, hipStream_t s);
// the marked plan if it is still alive (the mark stays)
const Plan *peek_internal(Buffer *adf_h, hipStream_t s);

// ---- halo exchange (halo_rccl.hip): enqueue pack -> grouped ncclSend/ncclRecv -> unpack on the
// halo plan's communication stream after the work already queued on `s`.  Returns an event that
// completes when the halo columns hold the neighbours' values (nullptr on failure).
// ntr tracers of plus/minus, `stride` doubles apart (the batched layouts)
hipEvent_t halo_exchange_async(void **comm, void **plan, Buffer *plus, Buffer *minus, int ntr, size_t stride,
                               hipStream_t s);

}  // namespace f2a
