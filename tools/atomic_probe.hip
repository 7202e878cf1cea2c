// atomic_probe.hip -- b1-horizontal as the reference writes it (edge -> node scatter with fp64 atomic
// adds, kernels/atomicAddFix.cu / src/fesom2-accelerate.cu's b1h launch, SURVEY.md 8(a) "fp64
// atomics") against the engine's ordered node gather, on the same structured mesh and the same
// fct_adf_h.  The engine's design rests on this comparison ("Gathers, not atomics"):
// this tool measures it instead of taking the guide's f32 atomic rate.
//
//   atomic   thread = (edge, level), 4 no-return global_atomic_add_f64 per cell into plus/minus of
//            both endpoints (plus/minus zeroed by hipMemsetAsync first, timed separately); a wave's
//            64 lanes add to 64 consecutive levels of one column: the coalesced shape, 512 B per
//            wave-instruction
//   gather   thread = (node, level), the node's incident edges in ascending edge order (the
//            reference's addition order), one store each of plus and minus
//
// It also runs the atomic form twice and counts the cells whose sums differ bit for bit between the
// runs (atomics commit in arrival order: fp64 addition is not associative).
// Build: hipcc --offload-arch=gfx950 -O3 -munsafe-fp-atomics -o tools/atomic_probe tools/atomic_probe.hip
// Run:   tools/atomic_probe [nx=1600] [ny=750] [L=80] [reps=10]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

__global__ __launch_bounds__(256) void k_scatter_atomic(const int2 *__restrict__ edges, const double *__restrict__ adf_h,
                                                        double *plus, double *minus, long ncell, int L)
{
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ncell) return;
    const long e = t / L;
    const int z = (int)(t - e * L);
    const int2 nn = edges[e];
    const double f = adf_h[t];
    const long a = (long)nn.x * L + z, b = (long)nn.y * L + z;
    atomicAdd(plus + a, fmax(0., f));
    atomicAdd(minus + a, fmin(0., f));
    atomicAdd(plus + b, fmax(0., -f));
    atomicAdd(minus + b, fmin(0., -f));
}

// node -> incident edges (ascending), code = edge << 1 | (node is the edge's second endpoint)
__global__ __launch_bounds__(256) void k_gather(const int *__restrict__ ptr, const int *__restrict__ code,
                                                const double *__restrict__ adf_h, double *__restrict__ plus,
                                                double *__restrict__ minus, long ncell, int L)
{
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ncell) return;
    const long n = t / L;
    const int z = (int)(t - n * L);
    double p = 0., m = 0.;
    for (int k = ptr[n]; k < ptr[n + 1]; k++) {
        const int c = code[k];
        const double f = adf_h[(long)(c >> 1) * L + z];
        if (c & 1) {
            p += fmax(0., -f);
            m += fmin(0., -f);
        } else {
            p += fmax(0., f);
            m += fmin(0., f);
        }
    }
    plus[t] = p;
    minus[t] = m;
}

static uint64_t splitmix(uint64_t &s)
{
    uint64_t z = (s += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

int main(int argc, char **argv)
{
    const int nx = argc > 1 ? atoi(argv[1]) : 1600, ny = argc > 2 ? atoi(argv[2]) : 750;
    const int L = argc > 3 ? atoi(argv[3]) : 80, reps = argc > 4 ? atoi(argv[4]) : 10;
    const long N = (long)nx * ny;
    // periodic structured triangulation: right, up and diagonal edge of every node (E = 3N), edge list
    // in ascending (n1, n2) order of creation
    std::vector<int2> edges;
    edges.reserve(3 * N);
    for (int j = 0; j < ny; j++)
        for (int i = 0; i < nx; i++) {
            const int n = j * nx + i, r = j * nx + (i + 1) % nx, u = ((j + 1) % ny) * nx + i,
                      d = ((j + 1) % ny) * nx + (i + 1) % nx;
            edges.push_back(make_int2(n, r));
            edges.push_back(make_int2(n, u));
            edges.push_back(make_int2(n, d));
        }
    const long E = (long)edges.size();
    std::vector<int> ptr(N + 1, 0), code(2 * E);
    for (long e = 0; e < E; e++) {
        ptr[edges[e].x + 1]++;
        ptr[edges[e].y + 1]++;
    }
    for (long n = 0; n < N; n++) ptr[n + 1] += ptr[n];
    std::vector<int> fill(ptr.begin(), ptr.end() - 1);
    for (long e = 0; e < E; e++) {  // ascending e per node: the reference's sum order
        code[fill[edges[e].x]++] = (int)(e << 1);
        code[fill[edges[e].y]++] = (int)(e << 1 | 1);
    }
    std::vector<double> h((size_t)E * L);
    uint64_t s = 43;
    for (auto &v : h) v = ((double)(splitmix(s) >> 11) * 0x1.0p-53 - 0.5) * 1e-3;

    int2 *d_edges;
    int *d_ptr, *d_code;
    double *d_h, *d_p, *d_m, *d_p2, *d_m2;
    const size_t cn = (size_t)N * L;
    CHECK(hipMalloc(&d_edges, E * sizeof(int2)));
    CHECK(hipMalloc(&d_ptr, (N + 1) * sizeof(int)));
    CHECK(hipMalloc(&d_code, 2 * E * sizeof(int)));
    CHECK(hipMalloc(&d_h, h.size() * sizeof(double)));
    for (double **p : {&d_p, &d_m, &d_p2, &d_m2}) CHECK(hipMalloc(p, cn * sizeof(double)));
    CHECK(hipMemcpy(d_edges, edges.data(), E * sizeof(int2), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_ptr, ptr.data(), (N + 1) * sizeof(int), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_code, code.data(), 2 * E * sizeof(int), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_h, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));

    hipEvent_t e0, e1, e2;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventCreate(&e2));
    const long ecell = E * L;
    const unsigned gb_e = (unsigned)((ecell + 255) / 256), gb_n = (unsigned)((cn + 255) / 256);
    auto run_atomic = [&](double *p, double *m, float *ms_zero, float *ms_add) {
        CHECK(hipEventRecord(e0, 0));
        CHECK(hipMemsetAsync(p, 0, cn * sizeof(double), 0));
        CHECK(hipMemsetAsync(m, 0, cn * sizeof(double), 0));
        CHECK(hipEventRecord(e1, 0));
        k_scatter_atomic<<<gb_e, 256>>>(d_edges, d_h, p, m, ecell, L);
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(e2, 0));
        CHECK(hipEventSynchronize(e2));
        CHECK(hipEventElapsedTime(ms_zero, e0, e1));
        CHECK(hipEventElapsedTime(ms_add, e1, e2));
    };
    float z = 0, a = 0, best_z = 1e9, best_a = 1e9, best_g = 1e9;
    for (int r = 0; r < reps; r++) {
        run_atomic(d_p, d_m, &z, &a);
        best_z = fminf(best_z, z);
        best_a = fminf(best_a, a);
        CHECK(hipEventRecord(e0, 0));
        k_gather<<<gb_n, 256>>>(d_ptr, d_code, d_h, d_p2, d_m2, cn, L);
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float g = 0;
        CHECK(hipEventElapsedTime(&g, e0, e1));
        best_g = fminf(best_g, g);
    }
    // determinism: two atomic runs bit for bit; gather vs atomic
    std::vector<double> pa(cn), pb(cn), pg(cn);
    run_atomic(d_p, d_m, &z, &a);
    CHECK(hipMemcpy(pa.data(), d_p, cn * sizeof(double), hipMemcpyDeviceToHost));
    run_atomic(d_p, d_m, &z, &a);
    CHECK(hipMemcpy(pb.data(), d_p, cn * sizeof(double), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(pg.data(), d_p2, cn * sizeof(double), hipMemcpyDeviceToHost));
    long run_diff = 0, vs_gather = 0;
    double max_rel = 0.;
    for (size_t i = 0; i < cn; i++) {
        run_diff += pa[i] != pb[i];
        if (pa[i] != pg[i]) {
            vs_gather++;
            if (pg[i] != 0.) max_rel = fmax(max_rel, fabs(pa[i] - pg[i]) / fabs(pg[i]));
        }
    }
    const double added = 4.0 * 8.0 * (double)ecell;               // bytes the atomics add
    const double alg = 8.0 * (double)ecell + 16.0 * (double)cn;    // adf_h read once + plus/minus written
    printf("{\"mesh\": \"%dx%d\", \"L\": %d, \"edges\": %ld, \"edge_cells\": %ld, \"node_cells\": %zu, "
           "\"atomic_ms\": %.4f, \"atomic_zero_ms\": %.4f, \"atomic_added_TBps\": %.3f, "
           "\"gather_ms\": %.4f, \"gather_alg_TBps\": %.3f, \"atomic_over_gather\": %.2f, "
           "\"atomic_cells_differing_between_two_runs\": %ld, \"atomic_cells_differing_from_gather\": %ld, "
           "\"max_rel_diff\": %.3e}\n",
           nx, ny, L, E, ecell, cn, best_a, best_z, added / (best_a * 1e-3) / 1e12, best_g,
           alg / (best_g * 1e-3) / 1e12, (best_a + best_z) / best_g, run_diff, vs_gather, max_rel);
    return 0;
}
