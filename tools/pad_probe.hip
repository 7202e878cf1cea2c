// pad_probe.hip -- does the relative placement of p1v's 15 streams in HBM change their rate?
//
// The engine's fields are separate hipMalloc'd arrays of equal size (768 MB at 1.2M x 80), so the
// base addresses of ttf, LO, hnode, ... differ by multiples of a large power of two times 3.  If
// the channel/bank hash maps element i of every stream to the same bank at once, the streams
// conflict.  This probe runs stream_probe.hip's p1v column pattern (11 reads + 4 writes per cell,
// G = 8 column blocks) with the arrays carved from one pool, array k starting at
// k * (size rounded up to 2 MB) + k * pad, for several pads, next to separately hipMalloc'd arrays
// (what the engine does; their address deltas are printed).
// Build: hipcc --offload-arch=gfx950 -O3 -o pad_probe tools/pad_probe.hip
// Run:   ./pad_probe [nodes=1200000] [L=80]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
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
    double *plus, *minus;
};

__device__ __forceinline__ d2 ld(const double *p) { return *reinterpret_cast<const d2 *>(p); }
__device__ __forceinline__ void st(double *p, d2 v) { *reinterpret_cast<d2 *>(p) = v; }

__device__ __forceinline__ int xcd_tile(int b, int G)
{
    const int q = G >> 3, r = G & 7, x = b & 7, k = b >> 3;
    return x * q + (x < r ? x : r) + k;
}

// stream_probe.hip's k_cols: 11 reads + 4 writes per cell (adf_v and del_v in place)
__global__ __launch_bounds__(1024) void k_cols(Arrays a, int nodes, int L, int G)
{
    const int S = L / 2, t = threadIdx.x, j = t / S, u = t - j * S;
    const int n = xcd_tile(blockIdx.x, gridDim.x) * G + j;
    if (j >= G || n >= nodes) return;
    const int z0 = 2 * u, nl = L + 1;
    const size_t b = (size_t)n * L + z0, ab = (size_t)n * nl + z0;
    d2 s = ld(a.ttf + b) + ld(a.LO + b) + ld(a.adfv + ab) + ld(a.ainv + ab) + ld(a.area + ab) + ld(a.hn + b) +
           ld(a.hnn + b) + ld(a.dv + b);
    const size_t e = (size_t)3 * n * L + z0;
    d2 h = ld(a.adfh + e) + ld(a.adfh + e + L) + ld(a.adfh + e + 2 * L);
    st(a.plus + b, s);
    st(a.minus + b, h);
    st(const_cast<double *>(a.adfv) + ab, s - h);
    st(const_cast<double *>(a.dv) + b, s + h);
}

// read-only variant: the same 11 reads, one 16-B store per 64 threads (no write streams)
__global__ __launch_bounds__(1024) void k_cols_r(Arrays a, int nodes, int L, int G)
{
    const int S = L / 2, t = threadIdx.x, j = t / S, u = t - j * S;
    const int n = xcd_tile(blockIdx.x, gridDim.x) * G + j;
    if (j >= G || n >= nodes) return;
    const int z0 = 2 * u, nl = L + 1;
    const size_t b = (size_t)n * L + z0, ab = (size_t)n * nl + z0;
    d2 s = ld(a.ttf + b) + ld(a.LO + b) + ld(a.adfv + ab) + ld(a.ainv + ab) + ld(a.area + ab) + ld(a.hn + b) +
           ld(a.hnn + b) + ld(a.dv + b);
    const size_t e = (size_t)3 * n * L + z0;
    d2 h = ld(a.adfh + e) + ld(a.adfh + e + L) + ld(a.adfh + e + 2 * L);
    if (s.x == 12345.678 && h.y == 1.) st(a.plus + b, s);  // never true: keeps the loads
}

int main(int argc, char **argv)
{
    const long nodes = argc > 1 ? atol(argv[1]) : 1200000;
    const int L = argc > 2 ? atoi(argv[2]) : 80;
    const long cn = nodes * L, cnl = nodes * (L + 1);
    // sizes in doubles, in the engine's allocation order
    const long sz[11] = {cn, cn, cnl, cnl, cnl, cn, cn, cn, 3 * cn, cn, cn};
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const double bytes = 8.0 * cn * (8 + 3 + 4), rbytes = 8.0 * cn * 11;
    const int G = 8, thr = ((G * (L / 2) + 63) / 64) * 64;
    const dim3 grid((unsigned)((nodes + G - 1) / G));
    auto assign = [](Arrays &a, double **p) {
        a.ttf = p[0], a.LO = p[1], a.adfv = p[2], a.ainv = p[3], a.area = p[4], a.hn = p[5], a.hnn = p[6];
        a.dv = p[7], a.adfh = p[8], a.plus = p[9], a.minus = p[10];
    };
    auto timeit = [&](Arrays a, bool ro) {
        auto launch = [&] {
            if (ro) hipLaunchKernelGGL(k_cols_r, grid, dim3(thr), 0, 0, a, (int)nodes, L, G);
            else hipLaunchKernelGGL(k_cols, grid, dim3(thr), 0, 0, a, (int)nodes, L, G);
        };
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
        return (ro ? rbytes : bytes) / (ms * 1e-3) / 1e12;
    };
    const int trials = argc > 3 ? atoi(argv[3]) : 1;
    for (int trial = 0; trial < trials; trial++) {  // separate hipMallocs (the engine's layout)
        // a spacer of a different size each trial: the arrays land on other physical pages
        void *spacer = nullptr;
        if (trial) CHECK(hipMalloc(&spacer, (size_t)trial * 37 * 1048576 + 4096));
        double *p[11];
        for (int k = 0; k < 11; k++) {
            CHECK(hipMalloc(&p[k], sz[k] * sizeof(double)));
            CHECK(hipMemset(p[k], 0, sz[k] * sizeof(double)));
        }
        printf("hipMalloc deltas (MB, mod 2MB in B):");
        for (int k = 1; k < 11; k++) {
            const long d = (long)((char *)p[k] - (char *)p[k - 1]);
            printf(" %.1f/%ld", d / 1048576.0, ((d % 2097152) + 2097152) % 2097152);
        }
        printf("\n");
        Arrays a;
        assign(a, p);
        const double rw = timeit(a, false), ro = timeit(a, true);
        printf("%-24s 11R+4W %6.2f TB/s   11R %6.2f TB/s\n", "separate hipMalloc", rw, ro);
        for (int k = 0; k < 11; k++) CHECK(hipFree(p[k]));
        if (spacer) CHECK(hipFree(spacer));
    }
    for (int trial = 0; trial < trials; trial++) {  // one pool, arrays back to back + k * 4352 B
        void *spacer = nullptr;
        if (trial) CHECK(hipMalloc(&spacer, (size_t)trial * 37 * 1048576 + 4096));
        long total = 0;
        for (int k = 0; k < 11; k++) total += ((sz[k] * 8 + 2097151) / 2097152) * 2097152 + 4352;
        char *pool;
        CHECK(hipMalloc(&pool, total));
        CHECK(hipMemset(pool, 0, total));
        double *p[11];
        long off = 0;
        for (int k = 0; k < 11; k++) {
            p[k] = reinterpret_cast<double *>(pool + off + k * 4352);
            off += ((sz[k] * 8 + 2097151) / 2097152) * 2097152;
        }
        Arrays a;
        assign(a, p);
        const double rw = timeit(a, false), ro = timeit(a, true);
        printf("%-24s 11R+4W %6.2f TB/s   11R %6.2f TB/s\n", "pool trial", rw, ro);
        fflush(stdout);
        CHECK(hipFree(pool));
        if (spacer) CHECK(hipFree(spacer));
    }
    if (trials > 1) return 0;
    const long pads[] = {0, 256, 4096, 12544, 65536, 262144, 1048576, 3 * 1048576 + 4352};
    long total = 0;
    for (int k = 0; k < 11; k++) total += ((sz[k] * 8 + 2097151) / 2097152) * 2097152;
    total += 11L * pads[sizeof(pads) / sizeof(pads[0]) - 1] + 2097152;
    char *pool;
    CHECK(hipMalloc(&pool, total));
    CHECK(hipMemset(pool, 0, total));
    for (long pad : pads) {
        double *p[11];
        long off = 0;
        for (int k = 0; k < 11; k++) {
            p[k] = reinterpret_cast<double *>(pool + off + k * pad);
            off += ((sz[k] * 8 + 2097151) / 2097152) * 2097152;
        }
        Arrays a;
        assign(a, p);
        const double rw = timeit(a, false), ro = timeit(a, true);
        char nm[64];
        snprintf(nm, sizeof nm, "pool, pad %ld B", pad);
        printf("%-24s 11R+4W %6.2f TB/s   11R %6.2f TB/s\n", nm, rw, ro);
        fflush(stdout);
    }
    CHECK(hipFree(pool));
    return 0;
}
