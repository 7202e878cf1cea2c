// f2a_host.hip -- host-side helpers shared by the C-ABI files: error reporting, handle
// validation, transfers, and the derived mesh plans (node->edge CSR in ascending edge order,
// node clusters) that the gather kernels run on.
#include "f2a_host.hpp"

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <map>
#include <mutex>
#include <tuple>
#include <unordered_map>

namespace f2a {

namespace {
std::mutex g_mutex;
int g_path = -1;
thread_local std::string g_last_error;
std::atomic<unsigned long> g_errors{0};
}  // namespace

int g_resident = 0;

void report(const char *fmt, ...)
{
    char msg[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(msg, sizeof msg, fmt, ap);
    va_end(ap);
    g_last_error = msg;
    g_errors++;
    fprintf(stderr, "fesom2-accelerate: %s\n", msg);
}

bool ok(hipError_t st, const char *what)
{
    if (st == hipSuccess) return true;
    report("HIP error \"%s\" in %s: %s", hipGetErrorName(st), what, hipGetErrorString(st));
    return false;
}

const char *last_error() { return g_last_error.c_str(); }

unsigned long error_count() { return g_errors.load(); }

int kernel_path()
{
    if (g_path < 0) {
        const char *p = getenv("FESOM2_PATH");
        g_path = (p && (!strcmp(p, "stepwise") || !strcmp(p, "1"))) ? 1
                 : (p && (!strcmp(p, "reference") || !strcmp(p, "2"))) ? 2
                                                                          : 0;
    }
    return g_path;
}

void set_kernel_path(int p) { g_path = (p == 1 || p == 2) ? p : 0; }


Buffer *buf(void **h, const char *name)
{
    if (!h || !*h) {
        report("null handle for %s", name);
        return nullptr;
    }
    Buffer *b = static_cast<Buffer *>(*h);
    if (b->magic != Buffer::kMagic) {
        report("invalid handle for %s (not created by this library)", name);
        return nullptr;
    }
    note_use(b, b->serial);
    return b;
}

Buffer *need(void **h, size_t bytes, const char *name)
{
    Buffer *b = buf(h, name);
    if (b && b->size < bytes) {
        report("%s holds %zu bytes, the call needs %zu", name, b->size, bytes);
        return nullptr;
    }
    if (b && b->pad < kAllocPad) {
        report("%s has no %zu bytes of slack behind its end (not allocated by this library)", name, kAllocPad);
        return nullptr;
    }
    return b;
}

hipStream_t stream_of(void **s)
{
    if (!s || !*s) return nullptr;
    return *static_cast<hipStream_t *>(*s);
}

Buffer *allocate(void *host, size_t bytes, bool create_event)
{
    auto *m = new Buffer;
    m->serial = track_object(m);
    m->host_pointer = host;
    m->size = bytes;
    // kAllocPad bytes of slack behind every array: the level-pair loads of odd-L columns read the
    // level after a column's last one (the next column's first, discarded), and for the last column
    // of an array that is the pad
    if (!ok(hipMalloc(&m->device_pointer, bytes + kAllocPad), "hipMalloc")) {
        untrack_object(m);
        delete m;
        return nullptr;
    }
    m->pad = kAllocPad;
    if (create_event) {
        if (!ok(hipEventCreateWithFlags(&m->event, hipEventDisableTiming), "hipEventCreate")) {
            (void)hipFree(m->device_pointer);
            untrack_object(m);
            delete m;
            return nullptr;
        }
        m->has_event = true;
    }
    return m;
}

bool h2d(Buffer *b, bool sync, hipStream_t s, bool record)
{
    if (!b->host_pointer || !b->size) return true;
    b->version++;
    if (sync) return ok(hipMemcpy(b->device_pointer, b->host_pointer, b->size, hipMemcpyHostToDevice), "H2D");
    if (!ok(hipMemcpyAsync(b->device_pointer, b->host_pointer, b->size, hipMemcpyHostToDevice, s), "H2D async"))
        return false;
    if (record && b->has_event) return ok(hipEventRecord(b->event, s), "hipEventRecord");
    return true;
}

bool d2h_async(Buffer *b, hipStream_t s)
{
    if (!b->host_pointer || !b->size) return true;
    return ok(hipMemcpyAsync(b->host_pointer, b->device_pointer, b->size, hipMemcpyDeviceToHost, s), "D2H async");
}

// The reference waits on the producers' upload events before its kernels (fesom2-accelerate.cu:293,
// :316, :326).  A captured stream may not wait on an event recorded outside the capture, so inside
// a capture the wait is recorded instead and fesom2_graph_launch_ issues it on the launch stream
// before every replay.
void wait_event(Buffer *b, hipStream_t s)
{
    if (!b->has_event) return;
    if (capturing(s)) {
        if (!defer_event_wait(b, s))
            report("stream captured outside fesom2_graph_begin_: the wait for a buffer event is dropped");
        return;
    }
    (void)hipStreamWaitEvent(s, b->event, 0);
}

bool check_levels(int nl, const char *who)
{
    if (nl < 2 || nl > 1025) {
        report("%s: nl = %d (needs 2 <= nl <= 1025)", who, nl);
        return false;
    }
    return true;
}

DeviceArrays::~DeviceArrays()
{
    for (void *p : ptrs) (void)hipFree(p);
}

void *DeviceArrays::alloc(size_t bytes)
{
    void *p = nullptr;
    if (!ok(hipMalloc(&p, std::max<size_t>(bytes, 8)), "hipMalloc(plan)")) return nullptr;
    ptrs.push_back(p);
    return p;
}

// ----------------------------------------------------------------------------- kernel timing

namespace {
struct TimedLaunch {
    std::string name;
    hipEvent_t start = nullptr, stop = nullptr;
};
std::atomic<bool> g_timing{false};  // read per launch without the mutex
std::string g_timing_only;  // fesom2_kernel_timing_only_: time only launches of this name (empty: all)
std::mutex g_tmutex;
std::vector<TimedLaunch *> g_pending;
struct Acc {
    long count = 0;
    double ms = 0.0;
};
std::map<std::string, Acc> g_acc;

void resolve_pending()
{
    for (TimedLaunch *t : g_pending) {
        float ms = 0.f;
        if (hipEventSynchronize(t->stop) == hipSuccess && hipEventElapsedTime(&ms, t->start, t->stop) == hipSuccess) {
            Acc &a = g_acc[t->name];
            a.count++;
            a.ms += ms;
        }
        (void)hipEventDestroy(t->start);
        (void)hipEventDestroy(t->stop);
        delete t;
    }
    g_pending.clear();
}
}  // namespace

bool timing_enabled(const char *name)
{
    if (!g_timing) return false;
    std::lock_guard<std::mutex> lock(g_tmutex);
    return g_timing_only.empty() || g_timing_only == name;
}

// ----------------------------------------------------------------------------- live objects

namespace {
std::mutex g_live_mutex;
std::unordered_map<const void *, uint64_t> g_live;
uint64_t g_next_serial = 1;
}  // namespace

uint64_t track_object(const void *p)
{
    std::lock_guard<std::mutex> lock(g_live_mutex);
    const uint64_t s = g_next_serial++;
    g_live[p] = s;
    return s;
}

void untrack_object(const void *p)
{
    std::lock_guard<std::mutex> lock(g_live_mutex);
    g_live.erase(p);
}

bool object_live(const void *p, uint64_t serial)
{
    std::lock_guard<std::mutex> lock(g_live_mutex);
    auto it = g_live.find(p);
    return it != g_live.end() && it->second == serial;
}

// ----------------------------------------------------------------------------- graph captures

namespace {
struct OpenCapture {
    hipStream_t origin = nullptr;
    unsigned long long id = 0;  // hipStreamGetCaptureInfo id, shared by streams forked into it
    CaptureLog log;
    bool orphaned = false;      // ended by another thread: the opening thread frees it
};
std::mutex g_cap_mutex;
std::vector<OpenCapture *> g_caps;
thread_local OpenCapture *t_cap = nullptr;  // the capture this thread opened

// this thread's open capture (g_cap_mutex held); forgets one another thread has ended
OpenCapture *my_capture()
{
    if (t_cap && t_cap->orphaned) {
        delete t_cap;
        t_cap = nullptr;
    }
    return t_cap;
}

// the open capture stream s belongs to (g_cap_mutex held), or nullptr
OpenCapture *capture_of(hipStream_t s)
{
    if (!s) return nullptr;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    if (hipStreamGetCaptureInfo(s, &st, &id) != hipSuccess || st != hipStreamCaptureStatusActive) return nullptr;
    for (OpenCapture *c : g_caps)
        if (c->id == id) return c;
    return nullptr;
}

void add_unique(std::vector<CapturedUse> &v, const void *p, uint64_t serial)
{
    for (const CapturedUse &u : v)
        if (u.p == p) return;
    v.push_back({p, serial});
}
}  // namespace

bool capturing(hipStream_t s)
{
    if (!s) return false;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &st) == hipSuccess && st == hipStreamCaptureStatusActive;
}

bool any_capture()
{
    std::lock_guard<std::mutex> lock(g_cap_mutex);
    return !g_caps.empty();
}

void note_use(const void *p, uint64_t serial)
{
    if (!t_cap) return;
    std::lock_guard<std::mutex> lock(g_cap_mutex);
    if (OpenCapture *c = my_capture()) add_unique(c->log.uses, p, serial);
}

bool defer_event_wait(Buffer *b, hipStream_t s)
{
    std::lock_guard<std::mutex> lock(g_cap_mutex);
    OpenCapture *c = capture_of(s);
    if (!c) return false;
    add_unique(c->log.waits, b, b->serial);
    add_unique(c->log.uses, b, b->serial);
    return true;
}

// the capture log's record of b's mark (g_cap_mutex held), created at the first access
static CapturedMark &mark_record(OpenCapture *c, Buffer *b, bool read)
{
    for (CapturedMark &m : c->log.marks)
        if (m.b == b) return m;
    CapturedMark m{b, b->serial, b->int_plan, b->int_serial};
    m.read_first = read;
    c->log.marks.push_back(m);
    return c->log.marks.back();
}

void mark_internal(Buffer *adf_h, const Plan *plan, hipStream_t s)
{
    if (s) {
        std::lock_guard<std::mutex> lock(g_cap_mutex);
        if (OpenCapture *c = capture_of(s)) {
            CapturedMark &m = mark_record(c, adf_h, false);
            m.written = true;
            m.final_mark = plan;
            m.final_serial = plan ? plan->serial : 0;
        }
    }
    adf_h->int_plan = plan;
    adf_h->int_serial = plan ? plan->serial : 0;
}

static void note_mark_read(Buffer *adf_h, hipStream_t s)
{
    if (!s) return;
    std::lock_guard<std::mutex> lock(g_cap_mutex);
    if (OpenCapture *c = capture_of(s)) (void)mark_record(c, adf_h, true);
}

bool has_internal(Buffer *adf_h, hipStream_t s)
{
    note_mark_read(adf_h, s);
    return adf_h->int_plan != nullptr;
}

const Plan *peek_internal(Buffer *adf_h, hipStream_t s)
{
    note_mark_read(adf_h, s);
    const void *p = adf_h->int_plan;
    return p && object_live(p, adf_h->int_serial) ? static_cast<const Plan *>(p) : nullptr;
}

bool marks_replayable(const CaptureLog &log)
{
    for (const CapturedMark &m : log.marks)
        if (m.read_first && object_live(m.b, m.serial) &&
            (m.b->int_plan != m.entry || m.b->int_serial != m.entry_serial)) {
            report("fesom2_graph_launch_: the graph first reads a phase mark on buffer %p (fct_adf_h, fct_adf_v or "
                   "del_ttf_advvert) and expects it %s by the phase-1 call that sets it, but it is %s now (run the "
                   "matching phase first, or capture both)",
                   (const void *)m.b, m.entry ? "marked" : "not marked", m.b->int_plan ? "marked" : "not marked");
            return false;
        }
    return true;
}

void marks_apply(const CaptureLog &log)
{
    for (const CapturedMark &m : log.marks)
        if (m.written && object_live(m.b, m.serial)) {
            m.b->int_plan = m.final_mark;
            m.b->int_serial = m.final_serial;
        }
}

bool capture_open(hipStream_t s)
{
    {
        std::lock_guard<std::mutex> lock(g_cap_mutex);
        if (my_capture()) return false;
    }
    auto *c = new OpenCapture;
    c->origin = s;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamGetCaptureInfo(s, &st, &c->id) != hipSuccess || st != hipStreamCaptureStatusActive) {
        delete c;
        return false;
    }
    std::lock_guard<std::mutex> lock(g_cap_mutex);
    g_caps.push_back(c);
    t_cap = c;
    return true;
}

bool capture_close(hipStream_t s, CaptureLog *log, bool *foreign)
{
    // the opening thread's thread-local pointer must not outlive the capture: a capture another
    // thread opened is only unregistered here and marked orphaned; that thread frees it
    *foreign = false;
    std::lock_guard<std::mutex> lock(g_cap_mutex);
    for (size_t k = 0; k < g_caps.size(); k++) {
        OpenCapture *c = g_caps[k];
        if (!s || c->origin != s) continue;
        // capturing changed no mark: put back what the captured calls wrote
        for (const CapturedMark &m : c->log.marks)
            if (m.written && object_live(m.b, m.serial)) {
                m.b->int_plan = m.entry;
                m.b->int_serial = m.entry_serial;
            }
        g_caps.erase(g_caps.begin() + k);
        if (c != t_cap) {
            c->orphaned = true;
            *foreign = true;
            return false;
        }
        *log = std::move(c->log);
        t_cap = nullptr;
        delete c;
        return true;
    }
    return false;
}

void timing_begin(const char *name, hipStream_t s, void **token)
{
    auto *t = new TimedLaunch;
    t->name = name;
    // default (system-scope) release.  Measured against a device-scope release
    // (hipEventReleaseToDevice, tuning build FESOM2_EVENT_FENCE=0): 127k x 47 the same within noise,
    // 1.2M x 80 1 % slower per pass with the device-scope events around p1v (profiles/r04/
    // r04f_sweep_eventfence_*.txt), so the default stays.
    const unsigned flags = knob("FESOM2_EVENT_FENCE", 1) ? hipEventDefault : hipEventReleaseToDevice;
    if (hipEventCreateWithFlags(&t->start, flags) != hipSuccess || hipEventCreateWithFlags(&t->stop, flags) != hipSuccess) {
        if (t->start) (void)hipEventDestroy(t->start);
        delete t;
        *token = nullptr;
        return;
    }
    (void)hipEventRecord(t->start, s);
    *token = t;
}

void timing_end(void *token, hipStream_t s)
{
    auto *t = static_cast<TimedLaunch *>(token);
    (void)hipEventRecord(t->stop, s);
    std::lock_guard<std::mutex> lock(g_tmutex);
    g_pending.push_back(t);
    if (g_pending.size() > 4096) resolve_pending();
}

}  // namespace f2a

extern "C" {

// Switching only flips the flag: the recorded events are resolved when the statistics are read (or
// reset), so a caller may time every k-th step without a host synchronisation in between.
void fesom2_kernel_timing_(int *on)
{
    f2a::g_timing = on && *on;
}

void fesom2_kernel_timing_only_(const char *name)
{
    std::lock_guard<std::mutex> lock(f2a::g_tmutex);
    f2a::g_timing_only = name ? name : "";
}

void fesom2_kernel_timing_reset_(void)
{
    std::lock_guard<std::mutex> lock(f2a::g_tmutex);
    f2a::resolve_pending();
    f2a::g_acc.clear();
}

// "name count total_ms\n" lines into buf (truncated to *len bytes incl. NUL); *len = bytes needed.
void fesom2_kernel_stats_(char *buf, int *len)
{
    std::lock_guard<std::mutex> lock(f2a::g_tmutex);
    f2a::resolve_pending();
    std::string out;
    char line[256];
    for (auto &kv : f2a::g_acc) {
        snprintf(line, sizeof line, "%s %ld %.6f\n", kv.first.c_str(), kv.second.count, kv.second.ms);
        out += line;
    }
    const int need = (int)out.size() + 1;
    if (buf && *len > 0) {
        const int n = std::min(*len - 1, (int)out.size());
        memcpy(buf, out.data(), n);
        buf[n] = 0;
    }
    *len = need;
}

}  // extern "C"

namespace f2a {

// ----------------------------------------------------------------------------- plans

// Packed b3h blocks: greedy over an edge list, separately for each range [bounds[i], bounds[i+1])
// (the exchange-overlap split keeps its interior / boundary descriptors); ends[i] = descriptors of
// ranges < i+1.  Returns false only if an edge cannot fit a block (unreachable, see cap).
static bool pack_edges(const std::vector<int4> &einfo, const std::vector<int> &bounds, int &cap,
                       std::vector<int2> &desc, std::vector<unsigned short> &off, std::vector<int> &ends)
{
    desc.clear();
    ends.clear();
    off.assign(einfo.size(), 0);
    const int cenv = knob("FESOM2_B3HP_CAP", kB3hPackSlots);  // level pairs per block (tuning build A/B)
    // at least one edge of the deepest kind per block (else no block could take it), and at most
    // 2048 pairs = a 1024-thread block at two slots per thread (the launch falls back to two slots
    // per thread whenever one slot per thread would need more than 1024 threads)
    int lmax = 0;
    for (const int4 &ei : einfo) lmax = std::max(lmax, ei.z);
    cap = std::max({64, (lmax + 1) / 2, std::min(cenv, 2048)});
    for (size_t part = 0; part + 1 < bounds.size(); part++) {
        int k = bounds[part];
        const int k_end = bounds[part + 1];
        while (k < k_end) {
            const int k0 = k;
            int slots = 0;
            while (k < k_end && k - k0 < kB3hPackEdges) {
                const int s = (einfo[k].z + 1) / 2;
                if (slots + s > cap) break;
                off[k] = (unsigned short)slots;
                slots += s;
                k++;
            }
            if (k == k0) return false;  // unreachable with cap >= ceil(lmax / 2); never loop forever
            desc.push_back(make_int2(k0, k - k0));
        }
        ends.push_back((int)desc.size());
    }
    return true;
}

// MeshPlanDev::b3p_* over p_edge_info: descriptors [0, b3p_nint) for the interior edges, the rest
// for the boundary ones
// slot count shared by every edge of einfo[e0, e1) if the greedy packing gave each of descriptors
// [d0, d1) the next P = min(kB3hPackEdges, cap / slots) of them (the last fewer), else 0
static int regular_slots(const std::vector<int4> &einfo, int e0, int e1, const std::vector<int2> &desc, int d0, int d1,
                         int cap)
{
    if (e1 <= e0) return 0;
    const int sl = (einfo[e0].z + 1) / 2;
    for (int k = e0; k < e1; k++)
        if ((einfo[k].z + 1) / 2 != sl) return 0;
    const int P = std::min(kB3hPackEdges, cap / sl);
    for (int k = d0; k < d1; k++)
        if (desc[k].x != e0 + (k - d0) * P || desc[k].y != std::min(P, e1 - desc[k].x)) return 0;
    return sl;
}

static bool build_b3h_pack(Plan *plan, MeshPlanDev &d, const std::vector<int4> &einfo, int n_int)
{
    std::vector<int2> desc;
    std::vector<unsigned short> off;
    std::vector<int> ends;
    if (!pack_edges(einfo, {0, n_int, (int)einfo.size()}, d.b3p_cap, desc, off, ends)) return false;
    d.b3p_slots_int = regular_slots(einfo, 0, n_int, desc, 0, ends[0], d.b3p_cap);
    d.b3p_slots_bnd = regular_slots(einfo, n_int, (int)einfo.size(), desc, ends[0], (int)desc.size(), d.b3p_cap);
    d.b3p_desc = plan->mem.upload(desc);
    d.b3p_off = plan->mem.upload(off);
    d.b3p_nint = ends[0];
    d.b3p_ndesc = (int)desc.size();
    return desc.empty() || (d.b3p_desc && d.b3p_off);
}

int pass_order(const Plan &plan, int ntr)
{
    const MeshPlanDev &d = plan.dev;
    const long long flux_bytes = (long long)ntr * d.n_edges * (d.nl - 1) * (long long)sizeof(real);
    const bool on = plan.cache_order >= 0 ? plan.cache_order == 1 : flux_bytes <= kCacheOrderBytes;
    return on ? (1 | 4 | 8) : 0;
}

// Row pairs (R = 2; the tuning build tries R rows) inside an ascending patch (`cur`, first position
// `base` of the processing order): the
// patch's runs of consecutive node numbers are its grid rows; each p1v block of G positions takes
// G/2 consecutive nodes of one row and the G - G/2 nodes right below them in the next row, so the
// vertical and diagonal edges between the two rows fall inside blocks too (structured 1.2M x 80:
// 29 % -> 53 % block-internal edges, which p1v limits and b3h then skips).  Two runs pair when both
// hold at least G nodes and the upper one's first node has a neighbour in the lower one, which
// aligns the lower row under the upper; the lower row's nodes left of that follow the pair.  A
// numbering without long rows (space-filling curves, scattered) keeps its ascending order.
static void row_pairs(std::vector<int> &cur, size_t base, int G, const std::vector<int> &ptr,
                      const std::vector<int> &other, int R = 2)
{
    if (G < R || R < 2 || cur.size() < 2) return;
    std::vector<std::pair<size_t, size_t>> runs;  // [begin, end) in cur
    size_t s0 = 0;
    for (size_t i = 1; i <= cur.size(); i++)
        if (i == cur.size() || cur[i] != cur[i - 1] + 1) {
            runs.emplace_back(s0, i);
            s0 = i;
        }
    std::vector<int> out;
    out.reserve(cur.size());
    const size_t g = (size_t)G;
    std::vector<size_t> take(R), k(R), lead(R);  // nodes per block from each row; cursors; lead ends
    for (int q = 0; q < R; q++) take[q] = g / R + ((size_t)q >= R - g % R ? 1 : 0);  // the odd ones below
    size_t r = 0;
    while (r < runs.size()) {
        const size_t a0 = runs[r].first, a1 = runs[r].second;
        bool grouped = false;
        bool long_rows = r + R <= runs.size();
        for (int q = 0; long_rows && q < R; q++) long_rows = runs[r + q].second - runs[r + q].first >= g;
        const size_t align = (g - (base + out.size()) % g) % g;  // the upper row up to the block grid
        if (long_rows && a0 + align < a1) {
            // each lower row aligned under the one above: the first neighbour, in the lower row, of
            // the upper row's first grouped node
            k[0] = a0 + align;
            bool ok = true;
            for (int q = 1; q < R && ok; q++) {
                const size_t b0 = runs[r + q].first, b1 = runs[r + q].second;
                const int v = cur[std::min(k[q - 1], runs[r + q - 1].second - 1)], B0 = cur[b0], nB = (int)(b1 - b0);
                int first = nB;
                for (int e = ptr[v]; e < ptr[v + 1]; e++)
                    if (other[e] >= B0 && other[e] < B0 + nB) first = std::min(first, other[e] - B0);
                ok = first < nB;
                k[q] = lead[q] = b0 + (size_t)first;
            }
            if (ok) {
                for (size_t t = a0; t < k[0]; t++) out.push_back(cur[t]);
                bool left = true;
                while (left) {
                    left = false;
                    for (int q = 0; q < R; q++) {
                        const size_t end = runs[r + q].second;
                        for (size_t t = 0; t < take[q] && k[q] < end; t++) out.push_back(cur[k[q]++]);
                        left = left || k[q] < end;
                    }
                }
                for (int q = 1; q < R; q++) out.insert(out.end(), cur.begin() + runs[r + q].first, cur.begin() + lead[q]);
                grouped = true;
                r += R;
            }
        }
        if (!grouped) {
            out.insert(out.end(), cur.begin() + a0, cur.begin() + a1);
            r += 1;
        }
    }
    cur.swap(out);
}

// Strips inside a patch (`cur`, ascending index order): on a row-structured numbering (runs of
// consecutive numbers = the patch's rows) every node gets a column coordinate x -- offsets along its
// run, each run anchored under the run above through the mesh (the lower-row neighbour of least
// index of an upper node sits at the upper node's x, as row_pairs aligns its pairs) -- and the patch
// is walked strip by strip (x in [k*W, (k+1)*W)), each strip top to bottom.  A batch's tiles then
// reuse the previous row of their strip (2 W nodes x ntracers tiles back with row pairs) instead of
// the previous row of the whole patch.  No-op unless most of the patch sits in runs of >= W nodes.
static void strip_order(std::vector<int> &cur, int W, const std::vector<int> &ptr, const std::vector<int> &other)
{
    if (W < 2 || cur.size() < (size_t)2 * W) return;
    std::vector<std::pair<size_t, size_t>> runs;
    size_t s0 = 0, in_long = 0;
    for (size_t i = 1; i <= cur.size(); i++)
        if (i == cur.size() || cur[i] != cur[i - 1] + 1) {
            runs.emplace_back(s0, i);
            if (i - s0 >= (size_t)W) in_long += i - s0;
            s0 = i;
        }
    if (runs.size() < 2 || 4 * in_long < 3 * cur.size()) return;
    const long kNone = std::numeric_limits<long>::min();
    std::vector<long> x(cur.size(), kNone);
    for (size_t t = runs[0].first; t < runs[0].second; t++) x[t] = (long)(t - runs[0].first);
    for (size_t r = 0; r + 1 < runs.size(); r++) {
        const size_t b0 = runs[r + 1].first, b1 = runs[r + 1].second;
        const int B0 = cur[b0], nB = (int)(b1 - b0);
        // anchors: each node of run r with a coordinate places its least neighbour in run r+1
        for (size_t t = runs[r].first; t < runs[r].second; t++) {
            if (x[t] == kNone) continue;
            const int v = cur[t];
            int first = nB;
            for (int e = ptr[v]; e < ptr[v + 1]; e++)
                if (other[e] >= B0 && other[e] < B0 + nB) first = std::min(first, other[e] - B0);
            if (first < nB && x[b0 + first] == kNone) x[b0 + first] = x[t];
        }
        // the rest of the run by offset from its first anchor (a run without one starts at 0)
        size_t a = b1;
        for (size_t t = b0; t < b1; t++)
            if (x[t] != kNone) {
                a = t;
                break;
            }
        const long xa = a < b1 ? x[a] : 0;
        if (a == b1) a = b0;
        for (size_t t = b0; t < b1; t++) x[t] = xa + (long)t - (long)a;
    }
    // stable order by (strip, run): floor division for strips left of the first row's start
    std::vector<size_t> idx(cur.size());
    for (size_t t = 0; t < idx.size(); t++) idx[t] = t;
    auto strip_of = [&](size_t t) { return x[t] >= 0 ? x[t] / W : -((-x[t] + W - 1) / W); };
    std::stable_sort(idx.begin(), idx.end(), [&](size_t p, size_t q) { return strip_of(p) < strip_of(q); });
    std::vector<int> out(cur.size());
    for (size_t t = 0; t < idx.size(); t++) out[t] = cur[idx[t]];
    cur.swap(out);
}

PlanShape plan_shape(bool batched)
{
    PlanShape s;
    const char *patch = getenv(batched ? "FESOM2_BATCH_PATCH" : "FESOM2_PATCH");
    if (patch) s.patch = std::max(1, atoi(patch));  // 0 or 1: index order
    if (batched) {
        const char *gs = getenv("FESOM2_BATCH_GROUP_SHIFT");
        const char *gc = getenv("FESOM2_BATCH_GROUP");
        if (!patch) s.patch = PlanShape::kAuto;
        s.gshift = gs ? atoi(gs) : PlanShape::kAuto;
        s.gcols = gc ? std::max(0, atoi(gc)) : 0;
        s.strip = knob("FESOM2_BATCH_STRIP", PlanShape::kAuto);  // tuning build: strip width (0 off)
    } else {
        // automatic (the large-partition rule of build_plan) unless the tuning build sets a shape
        s.gshift = knob("FESOM2_GROUP_SHIFT", PlanShape::kAuto);
        s.gcols = knob("FESOM2_GROUP", 0);
    }
    return s;
}

long long large_partition_cells()
{
    // plan option FESOM2_LARGE_CELLS (read when a plan is built): owned wet cells from which the
    // large-partition rules apply
    const char *v = getenv("FESOM2_LARGE_CELLS");
    return v ? std::max(0ll, atoll(v)) : (32ll << 20);
}

ResolvedShape resolve_shape(const PlanShape &shape, long long wet_cells, int nl)
{
    ResolvedShape r;
    const bool large = wet_cells >= large_partition_cells();
    // explicit columns per block: every column-group kernel must fit 1024 threads with its widest
    // shape (one level per thread: nl - 1 slots)
    r.gcols = (shape.gcols > 0 && shape.gcols * (nl - 1) <= 1024) ? shape.gcols : 0;
    r.gshift = r.gcols ? 0 : shape.gshift;
    if (r.gshift == PlanShape::kAuto) {
        // a large partition (>= 32M owned wet cells): smaller blocks -- the largest column count below
        // the natural one that keeps >= 90 % of the block's lanes busy -- taken in row pairs with
        // the stash.  Measured, 6 tracers at 1.2M x 80 (40 slots; 8 columns natural), one box, 3
        // interleaved rounds: 6 columns (240 of 256 lanes) 21.26 ms, 3: 21.52-21.67, 12: 21.65, 4:
        // 21.76, 7: 23.15, 8: 23.0-23.3; with row pairs + stash 6 columns 21.24, 4: 22.05, 8: 22.43.
        // One tracer: 6 columns in row pairs with the stash 4.06 ms against 4.14-4.17 with 8 in
        // single rows (-2.2 %), 6 columns alone -0.4 %.  On 127k x 47 (6M cells) every smaller
        // block loses (5 columns: +1.6 %, 7: +0.6 %): small partitions keep the natural one.
        r.gshift = 0;
        if (large) {
            r.large = true;
            const int S = p1v_slots(nl), Gn = p1v_group_columns(nl, 0);
            for (int g = Gn - 1; g >= 1; g--)
                if (10 * g * S >= 9 * ((g * S + 63) / 64 * 64) && g * (nl - 1) <= 1024) {
                    r.gcols = g;
                    break;
                }
        }
    }
    // nodes per patch: the shape's (plan options FESOM2_PATCH / FESOM2_BATCH_PATCH), else by
    // numbering (build_plan); the batched plan's default: 4096 when its blocks are smaller
    // (measured 1024..16384 at 6 x 1.2M x 80), else the single-tracer plan's choice
    // (127k x 47: 16384 best)
    r.patch = shape.patch == PlanShape::kAuto ? (r.gshift < 0 || r.gcols ? 4096 : 0) : shape.patch;
    // FESOM2_P1V_B3H: 1 on, 0 off, unset: on for large partitions -- measured 1.2M x 80 (96M
    // cells) -3.5 % per pass, 127k x 47 (6M cells, latency-bound) +2 %
    const char *ienv = getenv("FESOM2_P1V_B3H");
    r.internal = ienv ? atoi(ienv) != 0 : large;
    // strips inside the patches (batched plan of a large partition): off unless the tuning build
    // asks (FESOM2_BATCH_STRIP), see strip_order
    r.strip = shape.strip == PlanShape::kAuto ? 0 : std::max(0, shape.strip);
    // cluster unions (MeshPlanDev::cu_ptr) in row-pair blocks on small partitions: p1v stages each
    // block's union of cluster columns into LDS once instead of gathering every column's cluster.
    // Measured at 127k x 47 (24 level pairs; one set of buffers, interleaved): 6 tracers -2.3 to
    // -3.1 % per pass (p1v -4.4 %), 1 tracer -1.2 %; at 1.2M x 80 (large partitions) +9 to +50 % --
    // the LDS images cost occupancy there.  The cap keeps the images to 16 KB per block (21 columns at L =
    // 47: the 4 x 2 blocks' unions hold 22, the last one gathered from memory).  Plan option
    // FESOM2_P1V_UNION: 0 off, unset automatic (small partitions, L <= 64), > 0 on (the tuning
    // build: 1 or 2 also picks the kernel's LDS layout)
    const char *uenv = getenv("FESOM2_P1V_UNION");
    const int S = p1v_slots(nl);
    const bool want = uenv ? atoi(uenv) != 0 : (!large && nl - 1 <= 64);
    if (want) {
        const int G = p1v_group_columns(nl, r.gshift, r.gcols);
        r.union_cap = std::max(G, (int)(16384 / (2 * 2 * (size_t)S * sizeof(real))));
        if (const int k = knob("FESOM2_P1V_UNION_MAX", 0); k > 0) r.union_cap = std::max(G, k);
    }
    return r;
}

std::unique_ptr<Plan> build_plan(const HostMesh &m, int n_owned, int n_total, int n_edges,
                                 int n_csr, int nl, const PlanShape &shape, std::string &err)
{
    auto plan = std::make_unique<Plan>();
    // plan option FESOM2_NUM_KERNELS: the stepwise path stops phase 1 after that many reference
    // steps (the reference's NUM_KERNELS macro, src/fesom2-accelerate.cu:256; alg_state bisection)
    if (const char *nk = getenv("FESOM2_NUM_KERNELS")) plan->num_kernels = atoi(nk);
    // plan option FESOM2_CACHE_ORDER (pass_order): 0 off, 1 on, unset automatic
    if (const char *co = getenv("FESOM2_CACHE_ORDER")) plan->cache_order = atoi(co) ? 1 : 0;
    MeshPlanDev &d = plan->dev;
    d.n_owned = n_owned;
    d.n_total = n_total;
    d.n_edges = n_edges;
    d.nl = nl;
    long long wet_cells = 0;  // owned wet cells (the size rules of resolve_shape)
    if (m.nlev_nod)
        for (int v = 0; v < n_owned; v++) wet_cells += std::max(m.nlev_nod[v] - 1, 0);
    const ResolvedShape rs = resolve_shape(shape, wet_cells, nl);
    plan->shape = rs;
    plan->wet_cells = wet_cells;
    d.gshift = rs.gshift;
    d.gcols = rs.gcols;
    // a large partition: smaller blocks, row-pair blocks and the internal edges' raw flux kept in
    // LDS (row_pairs, MeshPlanDev::int_stash; tuning: FESOM2_ROWPAIR, FESOM2_P1V_STASH)
    const bool large_auto = rs.large;
    const int L = nl - 1;
    char msg[256];
    auto fail = [&](const char *s) {
        err = s;
        return std::unique_ptr<Plan>();
    };
    // ---- node -> edge CSR.  Filling it in ascending edge order reproduces the order in which the
    // reference's edge loops add into each node (reference.cpp:406-425).
    std::vector<int> lev(n_edges);
    std::vector<int> ptr((size_t)n_csr + 1, 0);
    for (int e = 0; e < n_edges; e++) {
        const int n1 = m.edges[2 * (size_t)e] - 1, n2 = m.edges[2 * (size_t)e + 1] - 1;
        const int el1 = m.edge_tri[2 * (size_t)e] - 1, el2 = m.edge_tri[2 * (size_t)e + 1] - 1;
        if (n1 < 0 || n1 >= n_total || n2 < 0 || n2 >= n_total) {
            snprintf(msg, sizeof msg, "edges(:,%d) = (%d,%d) outside 1..%d", e + 1, n1 + 1, n2 + 1, n_total);
            return fail(msg);
        }
        if (el1 < 0 || el1 >= m.n_elem_total || el2 < -1 || el2 >= m.n_elem_total) {
            snprintf(msg, sizeof msg, "edge_tri(:,%d) = (%d,%d) outside 1..%ld", e + 1, el1 + 1, el2 + 1,
                     m.n_elem_total);
            return fail(msg);
        }
        const int nl1 = m.nlev_elem[el1] - 1, nl2 = el2 >= 0 ? m.nlev_elem[el2] - 1 : 0;  // reference.cpp:412-414
        lev[e] = std::max(nl1, nl2);
        if (lev[e] > L || lev[e] < 0) {
            snprintf(msg, sizeof msg, "edge %d carries %d levels, nl-1 = %d", e + 1, lev[e], L);
            return fail(msg);
        }
        plan->lmax_edges = std::max(plan->lmax_edges, lev[e]);
        if (n1 < n_csr) ptr[n1 + 1]++;
        if (n2 < n_csr) ptr[n2 + 1]++;
    }
    for (int n = 0; n < n_csr; n++) ptr[n + 1] += ptr[n];
    std::vector<EdgeRef> refs(ptr[n_csr]);
    std::vector<int> other(ptr[n_csr]);
    {
        std::vector<int> pos(ptr.begin(), ptr.end() - 1);
        for (int e = 0; e < n_edges; e++) {
            const int n1 = m.edges[2 * (size_t)e] - 1, n2 = m.edges[2 * (size_t)e + 1] - 1;
            if (n1 < n_csr) {
                other[pos[n1]] = n2;
                refs[pos[n1]++] = {e, lev[e] << 1, n2};
            }
            if (n2 < n_csr) {
                other[pos[n2]] = n1;
                refs[pos[n2]++] = {e, (lev[e] << 1) | 1, n1};
            }
        }
    }
    d.edge_ptr = plan->mem.upload(ptr);
    d.edges = plan->mem.upload(refs);
    if (!d.edge_ptr || !d.edges) return fail("device allocation for the edge plan failed");

    // ---- clusters: the nodes of the elements around each owned node (reference.cpp:358-378
    // takes the bound over those elements' UV_rhs, which a2 built from their 3 nodes).
    std::vector<int> rptr, zdry;
    std::vector<RingRef> ring;
    const bool with_ring = m.elem_nodes && m.nie && m.nie_num;
    if (with_ring) {
        rptr.assign((size_t)n_owned + 1, 0);
        zdry.assign(n_owned, 0);
        ring.reserve((size_t)n_owned * 7);
        for (int n = 0; n < n_owned; n++) {
            const int ne = m.nie_num[n];
            if (ne < 1 || ne > m.dim) {
                snprintf(msg, sizeof msg, "nod_in_elem2D_num(%d) = %d outside 1..%d", n + 1, ne, m.dim);
                return fail(msg);
            }
            int zd = 1 << 30;
            const size_t start = ring.size();
            for (int k = 0; k < ne; k++) {
                const int e = m.nie[(size_t)n * m.dim + k] - 1;
                if (e < 0 || e >= m.n_elem_total) {
                    snprintf(msg, sizeof msg, "nod_in_elem2D(%d,%d) = %d outside 1..%ld", k + 1, n + 1, e + 1,
                             m.n_elem_total);
                    return fail(msg);
                }
                const int le = m.nlev_elem[e] - 1;
                zd = std::min(zd, le);
                for (int j = 0; j < 3; j++) {
                    const int v = m.elem_nodes[3 * (size_t)e + j] - 1;
                    if (v < 0 || v >= n_total) {
                        snprintf(msg, sizeof msg, "elem2D_nodes(%d,%d) = %d outside 1..%d", j + 1, e + 1, v + 1, n_total);
                        return fail(msg);
                    }
                    size_t q = start;
                    while (q < ring.size() && ring[q].node != v) q++;
                    if (q == ring.size())
                        ring.push_back({v, le});
                    else
                        ring[q].lev = std::max(ring[q].lev, le);
                }
            }
            zdry[n] = zd;
            rptr[n + 1] = (int)ring.size();
        }
        d.ring_ptr = plan->mem.upload(rptr);
        d.ring = plan->mem.upload(ring);
        d.zdry = plan->mem.upload(zdry);
        if (!d.ring_ptr || !d.ring || !d.zdry) return fail("device allocation for the cluster plan failed");
        plan->has_ring = true;
    }

    // ---- processing order.  The ABI fixes the memory layout (columns in the caller's node order);
    // the order in which the kernels VISIT nodes is free.  Greedy BFS patches of ~patch nodes
    // (seeded at the lowest unvisited node, grown over the owned-node graph) keep the cluster and
    // edge gathers of neighbouring columns close in time, i.e. in the XCD's L2, whatever the
    // numbering (a row-major 1600-wide grid puts the j+-1 neighbours ~9 MB apart otherwise).
    // Nodes inside a patch keep ascending index order.  Results do not depend on the order: each
    // node's sums run over its own CSR in ascending edge order.
    if (n_csr == n_owned && n_owned > 0 && m.nlev_nod) {
        // Patch order: a numbering with locality (median |n1 - n2| over the edges at most N/64, e.g.
        // row-major or space-filling-curve numbered meshes) keeps ascending index order inside
        // large patches -- adjacent positions are then adjacent in memory too; a scattered
        // numbering gets Cuthill-McKee order inside smaller patches (measured).
        bool local_numbering = true;
        {
            std::vector<int> gap;
            gap.reserve(refs.size());
            for (int n = 0; n < n_owned; n++)
                for (int k = ptr[n]; k < ptr[n + 1]; k++) gap.push_back(std::abs(other[k] - n));
            if (!gap.empty()) {
                std::nth_element(gap.begin(), gap.begin() + gap.size() / 2, gap.end());
                local_numbering = gap[gap.size() / 2] <= std::max(n_owned / 64, 64);
            }
        }
        // nodes per patch (1 = index order): the shape's (plan options FESOM2_PATCH /
        // FESOM2_BATCH_PATCH), else by numbering; the batched plan's default: 4096 when its blocks
        // are smaller (measured 1024..16384 at 6 x 1.2M x 80), else the single-tracer
        // plan's choice (127k x 47: 16384 best)
        const int patch = rs.patch > 0 ? rs.patch : (local_numbering ? 16384 : 4096);
        // order inside a patch: ascending index (0) or Cuthill-McKee (1); FESOM2_PATCH_ORDER in the
        // tuning build
        const int porder = knob("FESOM2_PATCH_ORDER", local_numbering ? 0 : 1);
        std::vector<int> order;
        // a union plan's row pairs serve p1v's blocks only: b3h's edge order and phase 2's node
        // records follow the patches' plain order (`plain`), which streams better for them (127k x 47:
        // row pairs cost b3h 2 % and p2h 1 %)
        std::vector<int> plain;
        std::vector<int> stamp, bq;  // FESOM2_PATCH_ORDER = 1: patch membership stamps, BFS queue
        if (porder == 1) stamp.assign(n_owned, -1);
        int npatch = 0;
        order.reserve(n_owned);
        if (patch <= 1) {
            for (int n = 0; n < n_owned; n++) order.push_back(n);
        } else {
            std::vector<char> seen(n_owned, 0);
            std::vector<int> queue, cur;
            int cursor = 0;
            while ((int)order.size() < n_owned) {
                while (seen[cursor]) cursor++;
                queue.assign(1, cursor);
                seen[cursor] = 1;
                cur.clear();
                for (size_t h = 0; h < queue.size() && (int)cur.size() < patch; h++) {
                    const int v = queue[h];
                    cur.push_back(v);
                    for (int k = ptr[v]; k < ptr[v + 1]; k++) {
                        const int w = other[k];
                        if (w < n_owned && !seen[w]) {
                            seen[w] = 1;
                            queue.push_back(w);
                        }
                    }
                }
                for (size_t h = cur.size(); h < queue.size(); h++) seen[queue[h]] = 0;  // back to the pool
                if (porder == 1 && cur.size() > 2) {
                    // Cuthill-McKee inside the patch from a peripheral node (the last node a BFS
                    // from the seed reaches): the BFS level sets cut across the patch, so graph
                    // neighbours sit at most about one patch width apart, whatever the numbering
                    const int id = npatch;
                    for (int v : cur) stamp[v] = id;
                    auto bfs = [&](int root) {
                        bq.assign(1, root);
                        stamp[root] = id + n_owned;  // visited mark for this sweep
                        for (size_t h = 0; h < bq.size(); h++)
                            for (int k = ptr[bq[h]]; k < ptr[bq[h] + 1]; k++) {
                                const int w = other[k];
                                if (w < n_owned && stamp[w] == id) {
                                    stamp[w] = id + n_owned;
                                    bq.push_back(w);
                                }
                            }
                        for (int v : bq) stamp[v] = id;
                    };
                    bfs(cur[0]);
                    if (bq.size() == cur.size()) {
                        bfs(bq.back());
                        cur.assign(bq.begin(), bq.end());
                    } else {
                        std::sort(cur.begin(), cur.end());
                    }
                    if (rs.union_cap > 0) plain.insert(plain.end(), cur.begin(), cur.end());
                } else {
                    std::sort(cur.begin(), cur.end());
                    if (rs.strip > 0) strip_order(cur, rs.strip, ptr, other);
                    if (rs.union_cap > 0) plain.insert(plain.end(), cur.begin(), cur.end());
                    // row pairs on large partitions, with the stash below (1.2M x 80: -2.2 % with 6
                    // columns, 6 tracers -1.2 %)
                    // (tuning: FESOM2_ROWPAIR = R > 1 takes R rows per block)
                    if (const int rp = knob("FESOM2_ROWPAIR", (large_auto || rs.union_cap > 0) ? 1 : 0))
                        row_pairs(cur, order.size(), p1v_group_columns(nl, d.gshift, d.gcols), ptr, other,
                                  rp > 1 ? rp : 2);
                }
                npatch++;
                order.insert(order.end(), cur.begin(), cur.end());
            }
        }
        std::vector<NodeInfo> info(n_owned);
        std::vector<EdgeRef> pedges;
        std::vector<RingRef> pring;
        pedges.reserve(refs.size());
        pring.reserve(ring.size());
        for (int k = 0; k < n_owned; k++) {
            const int n = order[k];
            NodeInfo &ni = info[k];
            ni.n = n;
            ni.Ln = m.nlev_nod[n] - 1;
            if (ni.Ln < 0 || ni.Ln > L) {
                snprintf(msg, sizeof msg, "nlevels_nod2D(%d) = %d outside 1..%d", n + 1, ni.Ln + 1, nl);
                return fail(msg);
            }
            ni.e0 = (int)pedges.size();
            pedges.insert(pedges.end(), refs.begin() + ptr[n], refs.begin() + ptr[n + 1]);
            ni.e1 = (int)pedges.size();
            ni.r0 = (int)pring.size();
            ni.self_lev = 0;
            if (with_ring) {  // the node itself last (k_p1 takes it from its own column, see RingRef)
                for (int r = rptr[n]; r < rptr[n + 1]; r++)
                    if (ring[r].node == n) ni.self_lev = ring[r].lev;
                    else pring.push_back(ring[r]);
                pring.push_back(RingRef{n, ni.self_lev});
            }
            ni.r1 = (int)pring.size();
            ni.zdry = with_ring ? zdry[n] : 0;
        }
        // the cluster union of every p1v block (ResolvedShape::union_cap; see MeshPlanDev::cu_ptr):
        // its own columns first, then the other cluster nodes in order of first use; each RingRef of
        // the processing-order copies gets its slot in the union above the level count.  Skipped
        // when a union would exceed the block's threads (one id each) or 64 KB of LDS images.
        if (with_ring && rs.union_cap > 0 && L <= kLevMask) {
            const int UG = p1v_group_columns(nl, d.gshift, d.gcols), S = p1v_slots(nl);
            // at most `cap` nodes per union (never fewer than the block's own columns): the cluster
            // nodes past it keep slot 0, and p1v gathers those from memory
            const int cap = std::max(UG, rs.union_cap);
            std::vector<int> sizes;
            const int nblk = (n_owned + UG - 1) / UG;
            std::vector<int> cptr(nblk + 1, 0), cnode;
            std::vector<RingRef> enc(pring);
            std::vector<int> slot_of_node(n_total, -1);
            int most = 0;
            for (int b = 0; b < nblk; b++) {
                const int k0 = b * UG, k1 = std::min(n_owned, k0 + UG);
                const size_t base = cnode.size();
                for (int k = k0; k < k1; k++) {
                    slot_of_node[info[k].n] = k - k0;
                    cnode.push_back(info[k].n);
                }
                for (int k = k0; k < k1; k++)
                    for (int r = info[k].r0; r < info[k].r1; r++) {
                        int &sl = slot_of_node[pring[r].node];
                        if (sl < 0 && (int)(cnode.size() - base) < cap) {
                            sl = (int)(cnode.size() - base);
                            cnode.push_back(pring[r].node);
                        }
                        enc[r].lev = pring[r].lev | (sl >= 0 ? (sl + 1) << kStashShift : 0);
                    }
                for (size_t q = base; q < cnode.size(); q++) slot_of_node[cnode[q]] = -1;
                cptr[b + 1] = (int)cnode.size();
                most = std::max(most, (int)(cnode.size() - base));
                sizes.push_back((int)(cnode.size() - base));
            }
            const int threads = (UG * S + 63) / 64 * 64;
            if (most <= threads && 2 * (size_t)most * 2 * S * sizeof(real) <= 65536) {
                pring.swap(enc);
                d.cu_G = UG;
                d.cu_max = most;
                d.cu_ptr = plan->mem.upload(cptr);
                d.cu_node = plan->mem.upload(cnode);
                if (!d.cu_ptr || !d.cu_node) return fail("device allocation for the cluster unions failed");
            }
            if (knob("FESOM2_PLAN_STATS", 0) && !sizes.empty()) {
                long outside = 0;
                for (const RingRef &rr : pring) outside += (rr.lev >> kStashShift) == 0;
                std::sort(sizes.begin(), sizes.end());
                fprintf(stderr, "fesom2-accelerate: p1v G=%d cluster unions: %zu nodes over %d blocks (p50 %d, p90 %d, "
                        "p99 %d, max %d; cap %d), %zu ring entries, %ld outside a union\n", UG, cnode.size(), nblk,
                        sizes[sizes.size() / 2], sizes[sizes.size() * 9 / 10], sizes[sizes.size() * 99 / 100], most,
                        cap, pring.size(), outside);
            }
        }
        // edges in the order of their first visited endpoint (edges without an owned endpoint last)
        std::vector<int4> einfo;
        einfo.reserve(n_edges);
        std::vector<char> etaken(n_edges, 0);
        auto push_edge = [&](int e) {
            etaken[e] = 1;
            einfo.push_back(make_int4(m.edges[2 * (size_t)e] - 1, m.edges[2 * (size_t)e + 1] - 1, lev[e], e));
        };
        if (plain.size() != order.size()) plain = order;  // (index order, or no union plan)
        for (int v : plain)
            for (int k = ptr[v]; k < ptr[v + 1]; k++)
                if (!etaken[refs[k].edge]) push_edge(refs[k].edge);
        for (int e = 0; e < n_edges; e++)
            if (!etaken[e]) push_edge(e);
        // interior / boundary split for the exchange overlap (stable: processing order kept), the
        // interior part split again into edges crossing p1v blocks and edges inside one p1v block
        // (both endpoints among the same int_G positions: p1v limits those itself, see int_ptr)
        auto interior_edge = [&](const int4 &ei) { return ei.x < n_owned && ei.y < n_owned; };
        std::stable_partition(einfo.begin(), einfo.end(), interior_edge);
        d.n_edge_interior = (int)std::count_if(einfo.begin(), einfo.end(), interior_edge);
        // FESOM2_P1V_B3H: 1 on, 0 off, unset: on from 32M owned wet cells per GPU -- measured
        // 1.2M x 80 (96M cells) -3.5 % per pass, 127k x 47 (6M cells, latency-bound) +2 %
        if (rs.internal) {
            const int IG = p1v_group_columns(nl, d.gshift, d.gcols);
            std::vector<int> pos(n_owned);
            for (int k = 0; k < n_owned; k++) pos[order[k]] = k;
            auto internal = [&](const int4 &ei) { return pos[ei.x] / IG == pos[ei.y] / IG; };
            // the interior edges crossing p1v blocks, in processing order (b3h's list on the split
            // path; p_edge_info keeps every edge in processing order for the other paths)
            std::vector<int4> ext;
            const int nblk = (n_owned + IG - 1) / IG;
            std::vector<int> iptr(nblk + 1, 0);
            for (int k = 0; k < d.n_edge_interior; k++) {
                if (internal(einfo[k])) iptr[pos[einfo[k].x] / IG + 1]++;
                else ext.push_back(einfo[k]);
            }
            int most = 0;
            for (int b = 0; b < nblk; b++) {
                most = std::max(most, iptr[b + 1]);
                iptr[b + 1] += iptr[b];
            }
            std::vector<int4> iedges(iptr[nblk]);
            std::vector<int> fill(iptr.begin(), iptr.end() - 1);
            for (int k = 0; k < d.n_edge_interior; k++) {
                const int4 ei = einfo[k];
                if (!internal(ei)) continue;
                const int b = pos[ei.x] / IG;
                // {edge, column of edges(1,e), column of edges(2,e), lev}: einfo keeps edges(1/2,e) order
                iedges[fill[b]++] = make_int4(ei.w, pos[ei.x] - b * IG, pos[ei.y] - b * IG, ei.z);
            }
            if (most <= kMaxInternal && nblk > 0 && !iedges.empty()) {
                std::vector<int2> xdesc;
                std::vector<unsigned short> xoff;
                std::vector<int> xends;
                int xcap = 0;
                if (!pack_edges(ext, {0, (int)ext.size()}, xcap, xdesc, xoff, xends))
                    return fail("packing the crossing edges failed");
                d.int_G = IG;
                d.int_max = most;
                for (const int4 &ie : iedges) plan->int_cells += ie.w;
                // the LDS stash (large partitions; tuning: FESOM2_P1V_STASH): mark each
                // internal edge's first-endpoint EdgeRef with its slot in the block's list, for the
                // NodeRecs and p_edges built below
                // (the slab is int_max x L doubles of LDS per block: kept to 16 KB, 6.4 KB at 1.2M x 80)
                if (knob("FESOM2_P1V_STASH", large_auto ? 1 : 0) && L <= kLevMask &&
                    (size_t)most * L * sizeof(real) <= 16384) {
                    for (int b = 0; b < nblk; b++)
                        for (int k = iptr[b]; k < iptr[b + 1]; k++) {
                            const int4 ie = iedges[k];  // {edge, column of edges(1,e), column of edges(2,e), lev}
                            const NodeInfo &n1 = info[b * IG + ie.y];
                            for (int q = n1.e0; q < n1.e1; q++)
                                if (pedges[q].edge == ie.x && !(pedges[q].code & 1))
                                    pedges[q].code |= (k - iptr[b] + 1) << kStashShift;
                        }
                    d.int_stash = 1;
                }
                d.int_ptr = plan->mem.upload(iptr);
                d.int_edges = plan->mem.upload(iedges);
                d.n_ext_interior = (int)ext.size();
                d.p_edge_ext = plan->mem.upload(ext);
                d.b3x_desc = plan->mem.upload(xdesc);
                d.b3x_off = plan->mem.upload(xoff);
                d.b3x_ndesc = (int)xdesc.size();
                d.b3x_cap = xcap;
                // regular packing (every block P consecutive edges): the b3h blocks then compute their
                // slice instead of loading a descriptor (checked against the descriptors themselves)
                d.b3x_slots = regular_slots(ext, 0, (int)ext.size(), xdesc, 0, (int)xdesc.size(), xcap);
                if (!d.int_ptr || !d.int_edges || (!ext.empty() && (!d.p_edge_ext || !d.b3x_desc || !d.b3x_off)))
                    return fail("device allocation for the internal edge lists failed");
            } else {  // nothing to gain, or a block with too many: every interior edge crosses
                d.n_ext_interior = d.n_edge_interior;
            }
            if (knob("FESOM2_PLAN_STATS", 0))
                fprintf(stderr, "fesom2-accelerate: p1v G=%d internal edges %d of %d interior (max %d per block)\n", IG,
                        d.n_edge_interior - d.n_ext_interior, d.n_edge_interior, most);
        } else {
            d.n_ext_interior = d.n_edge_interior;
        }
        std::vector<NodeRec> recs(n_owned);
        for (int k = 0; k < n_owned; k++) {
            NodeRec &r = recs[k];
            memset(&r, 0, sizeof r);
            r.info = info[k];
            for (int q = 0; q < kRecRing && info[k].r0 + q < info[k].r1; q++) r.ring[q] = pring[info[k].r0 + q];
            for (int q = 0; q < kRecEdge && info[k].e0 + q < info[k].e1; q++) r.edge[q] = pedges[info[k].e0 + q];
        }
        d.node_rec = plan->mem.upload(recs);

        std::vector<char> interior_node(n_owned, 1);
        for (int n = 0; n < n_owned; n++)
            for (int k = ptr[n]; k < ptr[n + 1]; k++)
                if (other[k] >= n_owned) interior_node[n] = 0;
        std::vector<NodeRec> p2(recs);
        if (plain != order) {  // phase 2 in the plain order (see `plain`)
            std::vector<int> at(n_owned);
            for (int k = 0; k < n_owned; k++) at[order[k]] = k;
            for (int k = 0; k < n_owned; k++) p2[k] = recs[at[plain[k]]];
        }
        std::stable_partition(p2.begin(), p2.end(), [&](const NodeRec &r) { return interior_node[r.info.n] != 0; });
        d.n_p2_interior = (int)std::count(interior_node.begin(), interior_node.end(), (char)1);
        for (int n = 0; n < n_owned; n++) d.max_degree = std::max(d.max_degree, ptr[n + 1] - ptr[n]);
        d.p2_rec = plan->mem.upload(p2);
        d.node_info = plan->mem.upload(info);
        d.p_edges = plan->mem.upload(pedges);
        d.p_ring = with_ring ? plan->mem.upload(pring) : nullptr;
        d.p_edge_info = plan->mem.upload(einfo);
        if (!d.node_info || !d.node_rec || !d.p2_rec || !d.p_edges || (with_ring && !d.p_ring) || !d.p_edge_info ||
            !build_b3h_pack(plan.get(), d, einfo, d.n_edge_interior))
            return fail("device allocation for the processing order failed");
    } else if (n_edges > 0) {
        std::vector<int4> einfo(n_edges);
        for (int e = 0; e < n_edges; e++)
            einfo[e] = make_int4(m.edges[2 * (size_t)e] - 1, m.edges[2 * (size_t)e + 1] - 1, lev[e], e);
        d.n_edge_interior = d.n_ext_interior = n_edges;
        d.p_edge_info = plan->mem.upload(einfo);
        if (!d.p_edge_info || !build_b3h_pack(plan.get(), d, einfo, n_edges))
            return fail("device allocation for the edge list failed");
    }
    return plan;
}

namespace {
using PlanKey = std::tuple<const void *, const void *, const void *, const void *, const void *,
                           const void *, const void *, int, int, int, int, int, bool>;
std::map<PlanKey, std::shared_ptr<Plan>> g_plans;

template <class T>
std::vector<T> fetch(Buffer *b, size_t count)
{
    std::vector<T> v(count);
    if (count) (void)hipMemcpy(v.data(), b->device_pointer, count * sizeof(T), hipMemcpyDeviceToHost);
    return v;
}
}  // namespace

const Plan *get_plan(const MeshHandles &h, int n_owned, int n_total, int n_edges, int nl,
                     bool with_ring, bool batched)
{
    std::lock_guard<std::mutex> lock(g_mutex);
    PlanKey key{h.edges, h.edge_tri, h.nlev_elem, with_ring ? h.elem_nodes : nullptr,
                with_ring ? h.nie : nullptr, with_ring ? h.nie_num : nullptr, h.nlev_nod,
                n_owned, n_total, n_edges, nl, with_ring ? h.dim : 0, batched};
    auto it = g_plans.find(key);
    if (it != g_plans.end()) return it->second.get();
    // a batched call whose shape resolves like an existing single-tracer plan's shares that plan (one
    // build, one set of device arrays; a graph capture after fesom2_prepare_mesh_ finds it either
    // way): compared with the shape the plan was built with, before any mesh array comes back
    PlanKey skey = key;
    std::get<12>(skey) = false;
    if (batched) {
        auto si = g_plans.find(skey);
        if (si != g_plans.end() && si->second->shape == resolve_shape(plan_shape(true), si->second->wet_cells, nl)) {
            g_plans[key] = si->second;
            return si->second.get();
        }
    }
    if (any_capture()) {  // building a plan copies with hipMemcpy, which would break an open capture
        report("a mesh plan would be built while a graph capture is open: run the sequence once (or "
               "fesom2_prepare_mesh_) before fesom2_graph_begin_");
        return nullptr;
    }
    if (h.edges->size < 2 * sizeof(int) * (size_t)n_edges || h.edge_tri->size < 2 * sizeof(int) * (size_t)n_edges) {
        report("edge handles hold fewer than myDim_edge2D = %d edges", n_edges);
        return nullptr;
    }
    HostMesh m;
    std::vector<int> edges = fetch<int>(h.edges, 2 * (size_t)n_edges);
    std::vector<int> etri = fetch<int>(h.edge_tri, 2 * (size_t)n_edges);
    m.n_elem_total = (long)(h.nlev_elem->size / sizeof(int));
    std::vector<int> nle = fetch<int>(h.nlev_elem, m.n_elem_total);
    m.edges = edges.data();
    m.edge_tri = etri.data();
    m.nlev_elem = nle.data();
    std::vector<int> en, nie, nnum, nln;
    if (h.nlev_nod && n_owned > 0) {
        if (h.nlev_nod->size < sizeof(int) * (size_t)n_owned) {
            report("nlevels_nod2D holds fewer than myDim_nod2D = %d entries", n_owned);
            return nullptr;
        }
        nln = fetch<int>(h.nlev_nod, n_owned);
        m.nlev_nod = nln.data();
    }
    if (with_ring) {
        if (h.elem_nodes->size < 3 * sizeof(int) * (size_t)m.n_elem_total) {
            report("elem2D_nodes holds fewer than 3 x %ld entries", m.n_elem_total);
            return nullptr;
        }
        if (h.nie->size < sizeof(int) * (size_t)h.dim * n_owned || h.nie_num->size < sizeof(int) * (size_t)n_owned) {
            report("nod_in_elem2D handles hold fewer than myDim_nod2D = %d columns", n_owned);
            return nullptr;
        }
        en = fetch<int>(h.elem_nodes, 3 * (size_t)m.n_elem_total);
        nie = fetch<int>(h.nie, (size_t)h.dim * n_owned);
        nnum = fetch<int>(h.nie_num, n_owned);
        m.elem_nodes = en.data();
        m.nie = nie.data();
        m.nie_num = nnum.data();
        m.dim = h.dim;
    }
    // no single-tracer plan yet: a batched call whose shape resolves like the single-tracer one
    // builds that plan and registers it for both
    bool share = false;
    if (batched && g_plans.find(skey) == g_plans.end()) {
        long long wet = 0;
        for (int v : nln) wet += std::max(v - 1, 0);
        share = resolve_shape(plan_shape(true), wet, nl) == resolve_shape(plan_shape(false), wet, nl);
    }
    std::string err;
    std::shared_ptr<Plan> plan = build_plan(m, n_owned, n_total, n_edges, n_owned, nl, plan_shape(batched && !share), err);
    if (!plan) {
        report("invalid mesh: %s", err.c_str());
        return nullptr;
    }
    plan->serial = track_object(plan.get());
    g_plans[key] = plan;
    if (share) g_plans[skey] = plan;
    return plan.get();
}



void drop_plans_of(const Buffer *b)
{
    std::lock_guard<std::mutex> lock(g_mutex);
    for (auto it = g_plans.begin(); it != g_plans.end();) {
        const PlanKey &k = it->first;
        if (std::get<0>(k) == b || std::get<1>(k) == b || std::get<2>(k) == b || std::get<3>(k) == b ||
            std::get<4>(k) == b || std::get<5>(k) == b || std::get<6>(k) == b) {
            untrack_object(it->second.get());
            it = g_plans.erase(it);
        } else {
            ++it;
        }
    }
}

}  // namespace f2a
