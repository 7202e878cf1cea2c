// odd_probe.hip -- what do 16-byte pair loads at 8-byte alignment cost for odd L?
//
// With L odd (FESOM2's CORE2 mesh: nl = 48), a node column n*L starts 16-byte aligned for even n
// and 8-byte aligned for odd n, so half the columns' level pairs straddle 16-byte boundaries.
// stream_probe.hip's column pattern (11 reads + 4 writes per cell) measured 4.94 TB/s at 127k x 47
// against 5.65 TB/s at 127k x 48.  This probe runs the L-stride streams of that pattern three ways:
//   mis    pairs (z0, z0+1) of the column, as the kernels do (8-byte aligned for odd n)
//   al     the 16-byte-aligned chunk containing the pair's first level (rounded down; timing bound)
//   shfl   al + the missing level taken from the next lane (__shfl_down), i.e. what an aligned odd-L
//          pair load would cost if done for real
// Build: hipcc --offload-arch=gfx950 -O3 -o odd_probe tools/odd_probe.hip
// Run:   ./odd_probe [nodes=126976] [L=47]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double d2 __attribute__((ext_vector_type(2), aligned(8)));

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

__device__ __forceinline__ int xcd_tile(int b, int G)
{
    const int q = G >> 3, r = G & 7, x = b & 7, k = b >> 3;
    return x * q + (x < r ? x : r) + k;
}

struct A {
    const double *in[8];  // ttf, LO, hnode, hnode_new, del_v, adf_h x 3 (L-stride)
    double *out[4];       // plus, minus, del_v, scratch
};

template <int MODE>
__device__ __forceinline__ d2 ldp(const double *p, size_t b, bool odd)
{
    if constexpr (MODE == 0) {
        return *reinterpret_cast<const d2 *>(p + b);
    } else {
        const d2 t = *reinterpret_cast<const d2 *>(p + (b & ~(size_t)1));
        if constexpr (MODE == 1) return t;
        const double nx = __shfl_down(t.x, 1);
        d2 r;
        r.x = odd ? t.y : t.x;
        r.y = odd ? nx : t.y;
        return r;
    }
}

template <int MODE>
__global__ __launch_bounds__(1024) void k_odd(A a, int nodes, int L, int G)
{
    const int S = (L + 1) / 2, t = threadIdx.x, j = t / S, u = t - j * S;
    const int n = xcd_tile(blockIdx.x, gridDim.x) * G + j;
    if (j >= G || n >= nodes) return;
    const int z0 = 2 * u < L - 1 ? 2 * u : L - 2;  // keep the pair inside the column
    const size_t b = (size_t)n * L + z0;
    const bool odd = b & 1;
    d2 s = ldp<MODE>(a.in[0], b, odd) + ldp<MODE>(a.in[1], b, odd) + ldp<MODE>(a.in[2], b, odd) +
           ldp<MODE>(a.in[3], b, odd) + ldp<MODE>(a.in[4], b, odd);
    const size_t e = (size_t)3 * n * L + z0;
    d2 h = ldp<MODE>(a.in[5], e, e & 1) + ldp<MODE>(a.in[5], e + L, (e + L) & 1) +
           ldp<MODE>(a.in[5], e + 2 * L, (e + 2 * L) & 1);
    if constexpr (MODE == 0) {
        *reinterpret_cast<d2 *>(a.out[0] + b) = s;
        *reinterpret_cast<d2 *>(a.out[1] + b) = h;
        *reinterpret_cast<d2 *>(a.out[2] + b) = s + h;
    } else {  // aligned stores: each lane writes the aligned chunk (timing only)
        const size_t q = b & ~(size_t)1;
        *reinterpret_cast<d2 *>(a.out[0] + q) = s;
        *reinterpret_cast<d2 *>(a.out[1] + q) = h;
        *reinterpret_cast<d2 *>(a.out[2] + q) = s + h;
    }
}

int main(int argc, char **argv)
{
    const long nodes = argc > 1 ? atol(argv[1]) : 126976;
    const int L = argc > 2 ? atoi(argv[2]) : 47;
    const long cn = nodes * L;
    A a;
    for (int k = 0; k < 8; k++) {
        double *p;
        const long n = (k == 5 ? 3 : 1) * cn + 2;
        CHECK(hipMalloc(&p, n * sizeof(double)));
        CHECK(hipMemset(p, 0, n * sizeof(double)));
        a.in[k] = p;
    }
    for (int k = 0; k < 4; k++) {
        CHECK(hipMalloc(&a.out[k], (cn + 2) * sizeof(double)));
        CHECK(hipMemset(a.out[k], 0, (cn + 2) * sizeof(double)));
    }
    const int G = 8, S = (L + 1) / 2, thr = ((G * S + 63) / 64) * 64;
    const dim3 grid((unsigned)((nodes + G - 1) / G));
    const double bytes = 8.0 * cn * (5 + 3 + 3);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const char *names[3] = {"mis (pairs at 8-B alignment)", "al (aligned chunks)", "shfl (aligned + shuffle)"};
    for (int round = 0; round < 2; round++)
        for (int mode = 0; mode < 3; mode++) {
            auto launch = [&] {
                if (mode == 0) hipLaunchKernelGGL(k_odd<0>, grid, dim3(thr), 0, 0, a, (int)nodes, L, G);
                if (mode == 1) hipLaunchKernelGGL(k_odd<1>, grid, dim3(thr), 0, 0, a, (int)nodes, L, G);
                if (mode == 2) hipLaunchKernelGGL(k_odd<2>, grid, dim3(thr), 0, 0, a, (int)nodes, L, G);
            };
            for (int w = 0; w < 3; w++) launch();
            CHECK(hipDeviceSynchronize());
            const int reps = 50;
            CHECK(hipEventRecord(e0));
            for (int r = 0; r < reps; r++) launch();
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            ms /= reps;
            printf("L=%d %-30s %8.4f ms %6.2f TB/s\n", L, names[mode], ms, bytes / (ms * 1e-3) / 1e12);
        }
    return 0;
}
