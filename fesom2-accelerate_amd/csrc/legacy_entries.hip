// legacy_entries.hip -- the reference's C++ convenience entries a1 / a2 / a1+a2 on gpuMemory handles
// (include/fesom2-accelerate-legacy.hpp; reference include/fesom2-accelerate.h:155-209,
// src/fesom2-accelerate.cu:42-112).
//
// They keep the reference kernels' own conventions (kernels/fct_ale_a1.cu, fct_ale_a2.cu: one column
// stride maxLevels for every array, a1 over z < nLevels, fmax/fmin), which are not those of the phase
// path (src/reference.cpp: node columns of nl-1 levels, a1 over z < nlev-1).  A wave per node /
// element, levels across its 64 lanes; every index is validated on the host before the launch (the
// reference has no status to return, so a failure is reported and nothing runs).
#include "../../include/fesom2-accelerate-legacy.hpp"
#include "f2a_device.hpp"
#include "f2a_host.hpp"

#include <algorithm>
#include <mutex>
#include <vector>

using namespace f2a;

namespace {

// kernels/fct_ale_a1.cu: max/min of the low-order and the old solution, levels z < nLevels(n)
__global__ __launch_bounds__(kBlock) void k_a1_legacy(int n_nodes, int stride, const int *__restrict__ nlev,
                                                      const real *__restrict__ lo, const real *__restrict__ ttf,
                                                      real *__restrict__ tmax, real *__restrict__ tmin)
{
    const int n = wave_item();
    if (n >= n_nodes) return;
    const size_t b = (size_t)n * stride;
    for (int z = threadIdx.x & 63; z < nlev[n]; z += kWave) {
        const real a = lo[b + z], t = ttf[b + z];
        tmax[b + z] = fmax(a, t);
        tmin[b + z] = fmin(a, t);
    }
}

// kernels/fct_ale_a2.cu: per element the max/min over its three nodes for z < nLevels(e) - 1, the
// (-1e3, +1e3) fill for nLevels(e) - 1 <= z < maxLevels - 1
__global__ __launch_bounds__(kBlock) void k_a2_legacy(int n_elem, int stride, const int *__restrict__ nlev,
                                                      const int *__restrict__ elem_nodes, double2 *__restrict__ uv,
                                                      const real *__restrict__ tmax, const real *__restrict__ tmin)
{
    const int e = wave_item();
    if (e >= n_elem) return;
    const size_t b = (size_t)e * stride;
    const size_t i0 = (size_t)(elem_nodes[3 * e] - 1) * stride, i1 = (size_t)(elem_nodes[3 * e + 1] - 1) * stride,
                 i2 = (size_t)(elem_nodes[3 * e + 2] - 1) * stride;
    const int top = nlev[e] - 1;
    for (int z = threadIdx.x & 63; z < stride - 1 || z < top; z += kWave) {
        if (z < top) {
            double2 v;
            v.x = fmax(fmax(tmax[i0 + z], tmax[i1 + z]), tmax[i2 + z]);
            v.y = fmin(fmin(tmin[i0 + z], tmin[i1 + z]), tmin[i2 + z]);
            uv[b + z] = v;
        } else {
            uv[b + z] = make_double2(-1.e+3, 1.e+3);
        }
    }
}

Buffer *handle(gpuMemory *g, const char *name)
{
    void *h = g;
    return buf(&h, name);
}

template <class T>
bool fetch(Buffer *b, std::vector<T> &v, size_t n)
{
    v.resize(n);
    return n == 0 || ok(hipMemcpy(v.data(), b->device_pointer, n * sizeof(T), hipMemcpyDeviceToHost), "D2H(check)");
}

// reference transferToDevice / transferToHost (src/fesom2-accelerate.cu): synchronous or on `s`
bool to_device(Buffer *b, bool sync, hipStream_t s, const char *name)
{
    if (!b->host_pointer) {
        report("%s: no host array bound to %s", "fct_ale_a*_accelerated", name);
        return false;
    }
    return h2d(b, sync, s, false);
}

bool to_host(Buffer *b, bool sync, hipStream_t s, const char *name)
{
    if (!b->host_pointer) {
        report("%s: no host array bound to %s", "fct_ale_a*_accelerated", name);
        return false;
    }
    if (sync)
        return ok(hipStreamSynchronize(s), "hipStreamSynchronize") &&
               ok(hipMemcpy(b->host_pointer, b->device_pointer, b->size, hipMemcpyDeviceToHost), "D2H");
    return d2h_async(b, s);
}

// The index arrays' validation is cached per (handle, live serial, upload version, sizes): a
// legacy call reads them back only the first time (after the call's stream has drained, so a
// non-blocking host stream still writing them is ordered before the read), not on every call as
// round 4 did (a synchronous copy that serialised the device).  A host that writes the device
// arrays itself, not through transfer_var_/fesom2_upload_, is outside this cache.
struct Validated {
    const Buffer *a, *b;
    uint64_t sa, va, sb, vb;
    long long n, stride, nodes;
    bool operator==(const Validated &o) const
    {
        return a == o.a && b == o.b && sa == o.sa && va == o.va && sb == o.sb && vb == o.vb && n == o.n &&
               stride == o.stride && nodes == o.nodes;
    }
};
std::mutex g_valid_mutex;
std::vector<Validated> g_valid;  // a handful of (mesh, shape) entries

bool cached_valid(const Validated &v)
{
    std::lock_guard<std::mutex> lock(g_valid_mutex);
    return std::find(g_valid.begin(), g_valid.end(), v) != g_valid.end();
}

void remember_valid(const Validated &v)
{
    std::lock_guard<std::mutex> lock(g_valid_mutex);
    if (std::find(g_valid.begin(), g_valid.end(), v) != g_valid.end()) return;
    if (g_valid.size() >= 64) g_valid.erase(g_valid.begin());
    g_valid.push_back(v);
}

// a1's arrays and levels: node columns of `stride` doubles, nLevels(n) <= stride
bool check_a1(const char *who, int stride, int n_nodes, Buffer *nlev, Buffer *tmax, Buffer *tmin, Buffer *lo,
              Buffer *ttf, hipStream_t s)
{
    if (stride < 1 || n_nodes < 0) {
        report("%s: maxLevels = %d, nNodes = %d", who, stride, n_nodes);
        return false;
    }
    const size_t col = sizeof(real) * (size_t)stride * n_nodes;
    for (Buffer *b : {tmax, tmin, lo, ttf})
        if (b->size < col) {
            report("%s: a node array holds %zu bytes, %d columns of %d levels need %zu", who, b->size, n_nodes, stride, col);
            return false;
        }
    if (nlev->size < sizeof(int) * (size_t)n_nodes) {
        report("%s: nLevels_nod2D holds fewer than nNodes = %d entries", who, n_nodes);
        return false;
    }
    const Validated key{nlev, nullptr, nlev->serial, nlev->version, 0, 0, n_nodes, stride, 0};
    if (cached_valid(key)) return true;
    std::vector<int> nl;
    // a cache miss reads the indices back: wait for the whole device, not only `s` -- the upload may
    // have been enqueued on another (non-blocking) stream, and a check of the old contents would
    // cache a pass under the new version (once per upload, so the cost stays small)
    (void)s;
    if (!ok(hipDeviceSynchronize(), "hipDeviceSynchronize") || !fetch(nlev, nl, n_nodes)) return false;
    for (int n = 0; n < n_nodes; n++)
        if (nl[n] > stride) {
            report("%s: nLevels_nod2D(%d) = %d exceeds maxLevels = %d", who, n + 1, nl[n], stride);
            return false;
        }
    remember_valid(key);
    return true;
}

// a2's arrays and indices: element columns of `stride` level pairs, nodes within tmax/tmin
bool check_a2(const char *who, int stride, int n_elem, Buffer *nlev, Buffer *en, Buffer *uv, Buffer *tmax,
              Buffer *tmin, hipStream_t s)
{
    if (stride < 1 || n_elem < 0) {
        report("%s: maxLevels = %d, nElements = %d", who, stride, n_elem);
        return false;
    }
    if (uv->size < 2 * sizeof(real) * (size_t)stride * n_elem) {
        report("%s: UV_rhs holds %zu bytes, %d elements of %d level pairs need %zu", who, uv->size, n_elem, stride,
               2 * sizeof(real) * (size_t)stride * n_elem);
        return false;
    }
    const long nodes = (long)(std::min(tmax->size, tmin->size) / (sizeof(real) * (size_t)stride));
    if (nlev->size < sizeof(int) * (size_t)n_elem || en->size < 3 * sizeof(int) * (size_t)n_elem) {
        report("%s: nLevels_elem / elementNodes hold fewer than nElements = %d entries", who, n_elem);
        return false;
    }
    const Validated key{nlev, en, nlev->serial, nlev->version, en->serial, en->version, n_elem, stride, nodes};
    if (cached_valid(key)) return true;
    std::vector<int> nl, nodes_of;
    (void)s;  // (the whole device: see check_a1)
    if (!ok(hipDeviceSynchronize(), "hipDeviceSynchronize") || !fetch(nlev, nl, n_elem) ||
        !fetch(en, nodes_of, 3 * (size_t)n_elem))
        return false;
    for (int e = 0; e < n_elem; e++) {
        if (nl[e] - 1 > stride) {
            report("%s: nLevels_elem(%d) = %d exceeds maxLevels + 1 = %d", who, e + 1, nl[e], stride + 1);
            return false;
        }
        for (int k = 0; k < 3; k++)
            if (nodes_of[3 * e + k] < 1 || nodes_of[3 * e + k] > nodes) {
                report("%s: elementNodes(%d,%d) = %d outside 1..%ld", who, k + 1, e + 1, nodes_of[3 * e + k], nodes);
                return false;
            }
    }
    remember_valid(key);
    return true;
}

bool launch_a1(int stride, int n_nodes, Buffer *nlev, Buffer *tmax, Buffer *tmin, Buffer *lo, Buffer *ttf,
               hipStream_t s)
{
    init_swizzle();
    if (n_nodes > 0)
        hipLaunchKernelGGL(k_a1_legacy, dim3(grid_for(n_nodes)), dim3(kBlock), 0, s, n_nodes, stride, dptr<int>(nlev),
                           dptr<real>(lo), dptr<real>(ttf), dptr<real>(tmax), dptr<real>(tmin));
    return ok(hipGetLastError(), "fct_ale_a1 (legacy)");
}

bool launch_a2(int stride, int n_elem, Buffer *nlev, Buffer *en, Buffer *uv, Buffer *tmax, Buffer *tmin,
               hipStream_t s)
{
    init_swizzle();
    if (n_elem > 0)
        hipLaunchKernelGGL(k_a2_legacy, dim3(grid_for(n_elem)), dim3(kBlock), 0, s, n_elem, stride, dptr<int>(nlev),
                           dptr<int>(en), reinterpret_cast<double2 *>(dptr<real>(uv)), dptr<real>(tmax),
                           dptr<real>(tmin));
    return ok(hipGetLastError(), "fct_ale_a2 (legacy)");
}

}  // namespace

extern "C" {

// reference src/fesom2-accelerate.cu:42-67
void fct_ale_a1_accelerated(const int maxLevels, const int nNodes, struct gpuMemory *nLevels_nod2D,
                            struct gpuMemory *fct_ttf_max, struct gpuMemory *fct_ttf_min,
                            struct gpuMemory *fct_low_order, struct gpuMemory *ttf, bool synchronous,
                            hipStream_t stream)
{
    const PhaseRange range("fct_ale_a1_accelerated");
    const char *who = "fct_ale_a1_accelerated";
    Buffer *bn = handle(nLevels_nod2D, "nLevels_nod2D"), *bx = handle(fct_ttf_max, "fct_ttf_max"),
           *bm = handle(fct_ttf_min, "fct_ttf_min"), *blo = handle(fct_low_order, "fct_low_order"),
           *bt = handle(ttf, "ttf");
    if (!bn || !bx || !bm || !blo || !bt || !check_a1(who, maxLevels, nNodes, bn, bx, bm, blo, bt, stream)) return;
    if (!to_device(blo, synchronous, stream, "fct_low_order") || !to_device(bt, synchronous, stream, "ttf")) return;
    if (!launch_a1(maxLevels, nNodes, bn, bx, bm, blo, bt, stream)) return;
    if (!to_host(bx, synchronous, stream, "fct_ttf_max")) return;
    (void)to_host(bm, synchronous, stream, "fct_ttf_min");
}

// reference src/fesom2-accelerate.cu:69-89
void fct_ale_a2_accelerated(const int maxLevels, const int nElements, struct gpuMemory *nLevels_elem,
                            struct gpuMemory *elementNodes, struct gpuMemory *UV_rhs,
                            struct gpuMemory *fct_ttf_max, struct gpuMemory *fct_ttf_min, bool synchronous,
                            hipStream_t stream)
{
    const PhaseRange range("fct_ale_a2_accelerated");
    const char *who = "fct_ale_a2_accelerated";
    Buffer *bn = handle(nLevels_elem, "nLevels_elem"), *be = handle(elementNodes, "elementNodes"),
           *bu = handle(UV_rhs, "UV_rhs"), *bx = handle(fct_ttf_max, "fct_ttf_max"),
           *bm = handle(fct_ttf_min, "fct_ttf_min");
    if (!bn || !be || !bu || !bx || !bm || !check_a2(who, maxLevels, nElements, bn, be, bu, bx, bm, stream)) return;
    if (!to_device(bx, synchronous, stream, "fct_ttf_max") || !to_device(bm, synchronous, stream, "fct_ttf_min"))
        return;
    if (!launch_a2(maxLevels, nElements, bn, be, bu, bx, bm, stream)) return;
    (void)to_host(bu, synchronous, stream, "UV_rhs");
}

// reference src/fesom2-accelerate.cu:91-112: a1 then a2 on the device, only UV_rhs goes back
void fct_ale_a1_a2_accelerated(const int maxLevels, const int nNodes, const int nElements,
                               struct gpuMemory *nLevels_nod2D, struct gpuMemory *nLevels_elem,
                               struct gpuMemory *elementNodes, struct gpuMemory *fct_ttf_max,
                               struct gpuMemory *fct_ttf_min, struct gpuMemory *fct_low_order,
                               struct gpuMemory *ttf, struct gpuMemory *UV_rhs, bool synchronous,
                               hipStream_t stream)
{
    const PhaseRange range("fct_ale_a1_a2_accelerated");
    const char *who = "fct_ale_a1_a2_accelerated";
    Buffer *bnn = handle(nLevels_nod2D, "nLevels_nod2D"), *bne = handle(nLevels_elem, "nLevels_elem"),
           *be = handle(elementNodes, "elementNodes"), *bx = handle(fct_ttf_max, "fct_ttf_max"),
           *bm = handle(fct_ttf_min, "fct_ttf_min"), *blo = handle(fct_low_order, "fct_low_order"),
           *bt = handle(ttf, "ttf"), *bu = handle(UV_rhs, "UV_rhs");
    if (!bnn || !bne || !be || !bx || !bm || !blo || !bt || !bu ||
        !check_a1(who, maxLevels, nNodes, bnn, bx, bm, blo, bt, stream) ||
        !check_a2(who, maxLevels, nElements, bne, be, bu, bx, bm, stream))
        return;
    if (!to_device(blo, synchronous, stream, "fct_low_order") || !to_device(bt, synchronous, stream, "ttf")) return;
    if (!launch_a1(maxLevels, nNodes, bnn, bx, bm, blo, bt, stream) ||
        !launch_a2(maxLevels, nElements, bne, be, bu, bx, bm, stream))
        return;
    (void)to_host(bu, synchronous, stream, "UV_rhs");
}

}  // extern "C"
