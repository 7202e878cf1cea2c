// stream_probe.hip -- ceiling of p1v's stream pattern on MI355X (no gathers, no arithmetic to speak of).
//
// p1v (fct_ale_kernels.hip k_p1<..., VERT>) reads 11.5 and writes 4 doubles per wet cell from 13
// arrays (ttf, LO, adf_v, area_inv, area, hnode, hnode_new, del_v, 3 x adf_h) and writes plus, minus,
// adf_v, del_v.  This probe moves the same bytes:
//   copy   flat 16-B/lane copy of one array (the guide's 6.29 TB/s float4 copy)
//   flat   13 reads + 4 writes per level pair, thread = pair, linear order
//   cols   the same in p1v's block shape: G = 8 columns x L/2 threads, XCD-swizzled tiles, the three
//          stride-nl arrays at nl = L+1 (8-byte aligned 16-B loads), adf_h as three columns per node
// Build: hipcc --offload-arch=gfx950 -O3 -o stream_probe tools/stream_probe.hip (build() does)
// Run:   ./stream_probe [nodes=1200000] [L=80] [--json|--text] [tracers]  (--json: one line with the copy
//        and the G = 8 column-pattern rates -- odd L: p1v's slot shape at the ABI stride --, which
//        bench.py reports beside the roofline; tracers > 1 adds the batched pattern, one line per
//        block shape and tile order, before it)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

typedef double d2 __attribute__((ext_vector_type(2), aligned(8)));

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

struct Arrays {
    const double *ttf, *LO, *adfv, *ainv, *area, *hn, *hnn, *dv, *adfh;
    double *plus, *minus, *adfv_o, *dv_o;
};

__device__ __forceinline__ d2 ld(const double *p) { return *reinterpret_cast<const d2 *>(p); }
__device__ __forceinline__ void st(double *p, d2 v) { *reinterpret_cast<d2 *>(p) = v; }

__global__ __launch_bounds__(256) void k_copy(const d2 *__restrict__ a, d2 *__restrict__ b, long n)
{
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) b[i] = a[i];
}

// thread = level pair i of the flat (Cn) arrays
__global__ __launch_bounds__(256) void k_flat(Arrays a, long npairs)
{
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npairs) return;
    const long b = 2 * i;
    d2 s = ld(a.ttf + b) + ld(a.LO + b) + ld(a.adfv + b) + ld(a.ainv + b) + ld(a.area + b) + ld(a.hn + b) +
           ld(a.hnn + b) + ld(a.dv + b);
    d2 h = ld(a.adfh + 3 * b) + ld(a.adfh + 3 * b + 2) + ld(a.adfh + 3 * b + 4);
    st(a.plus + b, s);
    st(a.minus + b, h);
    st(a.adfv_o + b, s - h);
    st(a.dv_o + b, s + h);
}

__device__ __forceinline__ int xcd_tile(int b, int G)
{
    const int q = G >> 3, r = G & 7, x = b & 7, k = b >> 3;
    return x * q + (x < r ? x : r) + k;
}

// p1v's shape: block = G columns x S = L/2 slots; node columns n*L, stride-nl arrays n*(L+1),
// adf_h: three edge columns per node (edge e = 3n + k, column e*L)
__global__ __launch_bounds__(1024) void k_cols(Arrays a, int nodes, int L, int G, int swz = 1)
{
    const int S = L / 2, t = threadIdx.x, j = t / S, u = t - j * S;
    const int n = (swz ? xcd_tile(blockIdx.x, gridDim.x) : (int)blockIdx.x) * G + j;
    if (j >= G || n >= nodes) return;
    const int z0 = 2 * u, nl = L + 1;
    const size_t b = (size_t)n * L + z0, ab = (size_t)n * nl + z0;
    d2 s = ld(a.ttf + b) + ld(a.LO + b) + ld(a.adfv + ab) + ld(a.ainv + ab) + ld(a.area + ab) + ld(a.hn + b) +
           ld(a.hnn + b) + ld(a.dv + b);
    const size_t e = (size_t)3 * n * L + z0;
    d2 h = ld(a.adfh + e) + ld(a.adfh + e + L) + ld(a.adfh + e + 2 * L);
    st(a.plus + b, s);
    st(a.minus + b, h);
    st(a.adfv_o + ab, s - h);
    st(a.dv_o + b, s + h);
}

// odd L as p1v runs it: S = (L+1)/2 slots, the last slot holds one level (its pair load starts a
// level early, inside the column).  `stride` = doubles between columns of the L-stride arrays
// (L: the ABI layout; L+1: padded, every column 16-byte aligned).  align = 1: parity-aware pairing
// of the L-stride arrays -- a column starting at 8 mod 16 gets its single-level slot first, so all
// its pair loads are 16-byte aligned (the stride-nl arrays keep the plain pairing).
__device__ __forceinline__ d2 ld2(const double *p, bool single_hi, bool single_lo)
{
    if (single_lo) return d2{p[0], 0.0};
    return single_hi ? d2{0.0, p[1]} : ld(p);
}

__global__ __launch_bounds__(1024) void k_cols_odd(Arrays a, int nodes, int L, int G, int stride, int align)
{
    const int S = (L + 1) / 2, t = threadIdx.x, j = t / S, u = t - j * S;
    const int n = xcd_tile(blockIdx.x, gridDim.x) * G + j;
    if (j >= G || n >= nodes) return;
    const int nl = L + 1;
    const size_t col = (size_t)n * stride;
    const bool shifted = align && (col & 1);
    // L-stride arrays: plain pairs (2u, 2u+1), last slot = (L-2, L-1) taking the second; shifted:
    // slot 0 = level 0 alone, slot u = (2u-1, 2u)
    int zl;
    bool hi = false, lo = false;
    if (!shifted) {
        zl = 2 * u;
        if (zl + 1 == L) {
            zl -= 1;
            hi = true;
        }
    } else {
        zl = u == 0 ? 0 : 2 * u - 1;
        lo = u == 0;
    }
    int zn = 2 * u;  // stride-nl arrays: plain pairs, the last one at L-1 (nl = L+1 holds it)
    const size_t b = col + zl, ab = (size_t)n * nl + zn;
    d2 s = ld2(a.ttf + b, hi, lo) + ld2(a.LO + b, hi, lo) + ld(a.adfv + ab) + ld(a.ainv + ab) + ld(a.area + ab) +
           ld2(a.hn + b, hi, lo) + ld2(a.hnn + b, hi, lo) + ld2(a.dv + b, hi, lo);
    const size_t e = (size_t)3 * col + zl;
    d2 h = ld2(a.adfh + e, hi, lo) + ld2(a.adfh + e + stride, hi, lo) + ld2(a.adfh + e + 2 * stride, hi, lo);
    if (lo) {
        a.plus[b] = s.x;
        a.minus[b] = h.x;
        a.dv_o[b] = s.x + h.x;
    } else if (hi) {
        a.plus[b + 1] = s.y;
        a.minus[b + 1] = h.y;
        a.dv_o[b + 1] = s.y + h.y;
    } else {
        st(a.plus + b, s);
        st(a.minus + b, h);
        st(a.dv_o + b, s + h);
    }
    st(a.adfv_o + ab, s - h);
}

// batched tracers (fct_ale_pre_comm_v_acc_ with ntracers > 1): T tracers' own arrays (ttf, LO,
// adf_v, del_v, 3 x adf_h read; plus, minus, adf_v, del_v written) tracer k at offset k * tstride, the
// mesh fields (area_inv, area at stride nl; hnode, hnode_new) shared; tile -> (column group,
// tracer), tracer fastest (the product's p1v order) or slowest (major = 1)
__global__ __launch_bounds__(1024) void k_cols_batch(Arrays a, int nodes, int L, int G, int T, size_t tstride,
                                                     int major)
{
    const int S = L / 2, t = threadIdx.x, j = t / S, u = t - j * S;
    const int tile = xcd_tile(blockIdx.x, gridDim.x);
    int g, tr;
    if (major) {
        const int groups = gridDim.x / T;
        tr = tile / groups;
        g = tile - tr * groups;
    } else {
        g = tile / T;
        tr = tile - g * T;
    }
    const int n = g * G + j;
    if (j >= G || n >= nodes) return;
    const int z0 = 2 * u, nl = L + 1;
    const size_t o = (size_t)tr * tstride, b = (size_t)n * L + z0, ab = (size_t)n * nl + z0;
    d2 s = ld(a.ttf + o + b) + ld(a.LO + o + b) + ld(a.adfv + o + ab) + ld(a.ainv + ab) + ld(a.area + ab) +
           ld(a.hn + b) + ld(a.hnn + b) + ld(a.dv + o + b);
    const size_t e = o * 3 + (size_t)3 * n * L + z0;
    d2 h = ld(a.adfh + e) + ld(a.adfh + e + L) + ld(a.adfh + e + 2 * L);
    st(a.plus + o + b, s);
    st(a.minus + o + b, h);
    st(a.adfv_o + o + ab, s - h);
    st(a.dv_o + o + b, s + h);
}

int main(int argc, char **argv)
{
    const long nodes = argc > 1 ? atol(argv[1]) : 1200000;
    const int L = argc > 2 ? atoi(argv[2]) : 80;
    const bool json = argc > 3 && std::string(argv[3]) == "--json";  // "--text" (or anything else): a table
    double copy_tbs = 0, cols_tbs = 0;
    const long cn = nodes * L, cnl = nodes * (L + 1);
    std::vector<double *> bufs;
    // every array staggered by k x 4352 B from its allocation's start: separately hipMalloc'd
    // equal-size arrays start on 2 MB boundaries, so element i of each has the same low address bits
    // and the pattern's streams alias HBM channels -- it then moves 10-15 % less depending on where
    // the allocator put them (tools/pad_probe.hip): the staggered layout is the stable,
    // best-placement rate, i.e. the ceiling
    auto alloc = [&](long n) {
        double *p;
        const size_t skew = ((size_t)bufs.size() * 4352) % 65536;
        CHECK(hipMalloc(&p, n * sizeof(double) + 65536));
        CHECK(hipMemset(p, 0, n * sizeof(double) + 65536));
        bufs.push_back(p);
        return p + skew / sizeof(double);
    };
    Arrays a;
    a.ttf = alloc(cnl);  // room for the padded-stride variant
    a.LO = alloc(cnl);  // room for the padded-stride variant
    a.adfv = alloc(cnl);
    a.ainv = alloc(cnl);
    a.area = alloc(cnl);
    a.hn = alloc(cnl);  // room for the padded-stride variant
    a.hnn = alloc(cnl);  // room for the padded-stride variant
    a.dv = alloc(cnl);  // room for the padded-stride variant
    a.adfh = alloc(3 * cnl);
    a.plus = alloc(cnl);  // room for the padded-stride variant
    a.minus = alloc(cnl);  // room for the padded-stride variant
    a.adfv_o = const_cast<double *>(a.adfv);  // in place, as p1v
    a.dv_o = const_cast<double *>(a.dv);
    double *src = alloc(4 * cn), *dst = alloc(4 * cn);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const double bytes_p1 = 8.0 * cn * (8 + 3 + 4);  // 8 own + 3 adf_h reads, 4 writes per cell
    auto timeit = [&](const char *name, double bytes, auto launch) {
        for (int w = 0; w < 3; w++) launch();
        CHECK(hipDeviceSynchronize());
        const int reps = 20;
        CHECK(hipEventRecord(e0));
        for (int r = 0; r < reps; r++) launch();
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        const double tbs = bytes / (ms * 1e-3) / 1e12;
        if (!json) printf("%-28s %8.3f ms  %7.1f GB  %6.2f TB/s\n", name, ms, bytes / 1e9, tbs);
        fflush(stdout);
        return tbs;
    };
    const long n2 = 2 * cn;  // d2 elements of the copy
    copy_tbs = timeit("copy (16 B/lane)", 2.0 * 16 * n2, [&] {
        hipLaunchKernelGGL(k_copy, dim3((unsigned)((n2 + 255) / 256)), dim3(256), 0, 0, (const d2 *)src, (d2 *)dst, n2);
    });
    const long np = cn / 2;
    if (!json)
        timeit("flat 11R+4W", bytes_p1, [&] {
            hipLaunchKernelGGL(k_flat, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, 0, a, np);
        });
    for (int G : {4, 8, 16, 24}) {
        if (json && (G != 8 || L % 2 == 1)) continue;
        char nm[64];
        snprintf(nm, sizeof nm, "cols G=%d 11R+4W", G);
        const int thr = ((G * (L / 2) + 63) / 64) * 64;
        const double r = timeit(nm, bytes_p1, [&] {
            hipLaunchKernelGGL(k_cols, dim3((unsigned)((nodes + G - 1) / G)), dim3(thr), 0, 0, a, (int)nodes, L, G);
        });
        if (G == 8) cols_tbs = r;
    }
    if (L % 2 == 1) {  // odd L: p1v's slot shape, ABI stride vs padded vs parity-aware pairs
        const int G = 8, S = (L + 1) / 2, thr = ((G * S + 63) / 64) * 64;
        for (int mode = 0; mode < 3; mode++) {
            if (json && mode != 0) continue;
            const char *nm[3] = {"odd cols stride L", "odd cols stride L+1", "odd cols aligned pairs"};
            const int stride = mode == 1 ? L + 1 : L;
            const double r = timeit(nm[mode], bytes_p1, [&] {
                hipLaunchKernelGGL(k_cols_odd, dim3((unsigned)((nodes + G - 1) / G)), dim3(thr), 0, 0, a, (int)nodes, L,
                                   G, stride, mode == 2 ? 1 : 0);
            });
            if (mode == 0) cols_tbs = r;  // --json: p1v's own shape at odd L (the ABI stride)
        }
    }
    if (!json) {  // the same without the XCD-contiguous tile ranges (block b -> tile b)
        const int G = 8, thr = ((G * (L / 2) + 63) / 64) * 64;
        timeit("cols G=8 no XCD swizzle", bytes_p1, [&] {
            hipLaunchKernelGGL(k_cols, dim3((unsigned)((nodes + G - 1) / G)), dim3(thr), 0, 0, a, (int)nodes, L, G, 0);
        });
    }
    // --tracers T (4th argument): the batched pattern at G = 6 and 8 columns, tracer fastest/slowest
    const int T = argc > 4 ? atoi(argv[4]) : 0;
    if (T > 1 && L % 2 == 0) {
        Arrays bt = a;
        const size_t ts = (size_t)cnl;
        bt.ttf = alloc(T * cnl);
        bt.LO = alloc(T * cnl);
        bt.adfv = alloc(T * cnl);
        bt.dv = alloc(T * cnl);
        bt.adfh = alloc(3 * T * cnl);
        bt.plus = alloc(T * cnl);
        bt.minus = alloc(T * cnl);
        bt.adfv_o = const_cast<double *>(bt.adfv);
        bt.dv_o = const_cast<double *>(bt.dv);
        const double bytes_b = 8.0 * cn * (4 + T * (4 + 3 + 4));  // shared 4 reads; per tracer 7 reads + 4 writes
        for (int G : {6, 8})
            for (int major = 0; major < 2; major++) {
                char nm[64];
                snprintf(nm, sizeof nm, "batch T=%d G=%d %s", T, G, major ? "tracer-slowest" : "tracer-fastest");
                const int thr = ((G * (L / 2) + 63) / 64) * 64;
                const unsigned groups = (unsigned)((nodes + G - 1) / G);
                const double r = timeit(nm, bytes_b, [&] {
                    hipLaunchKernelGGL(k_cols_batch, dim3(groups * T), dim3(thr), 0, 0, bt, (int)nodes, L, G, T, ts, major);
                });
                if (json)
                    printf("{\"batch_GBps\": %.1f, \"tracers\": %d, \"G\": %d, \"order\": \"%s\"}\n", r * 1e3, T, G,
                           major ? "tracer-slowest" : "tracer-fastest");
            }
    }
    if (json)
        printf("{\"copy_GBps\": %.1f, \"p1v_pattern_GBps\": %.1f, \"nodes\": %ld, \"levels\": %d}\n", copy_tbs * 1e3,
               cols_tbs * 1e3, nodes, L);
    for (double *p : bufs) CHECK(hipFree(p));
    return 0;
}
