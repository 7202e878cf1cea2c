// xcc_probe.hip -- records which XCD (HW_REG_XCC_ID) each workgroup of a grid runs on, to check the
// round-robin block->XCD placement the kernels' swizzle assumes (MI355X_MICROARCH.md "Workgroup
// dispatch").  Diagnostic tool only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void probe(int *xcc)
{
    if (threadIdx.x == 0) {
        unsigned v;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
        xcc[blockIdx.x] = (int)(v & 0xf);
    }
}

int main(int argc, char **argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 4096;
    const int threads = argc > 2 ? atoi(argv[2]) : 320;
    int *d;
    hipMalloc(&d, n * sizeof(int));
    hipLaunchKernelGGL(probe, dim3(n), dim3(threads), 0, 0, d);
    std::vector<int> h(n);
    hipMemcpy(h.data(), d, n * sizeof(int), hipMemcpyDeviceToHost);
    int match = 0;
    for (int b = 0; b < n; b++) match += (h[b] == (h[b % 8]));
    printf("blocks %d threads %d: xcc(b) == xcc(b %% 8) for %d of %d blocks; first 24:", n, threads, match, n);
    for (int b = 0; b < 24; b++) printf(" %d", h[b]);
    printf("\n");
    return 0;
}
