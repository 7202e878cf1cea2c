// fesom2-accelerate-legacy.hpp -- the reference's C++ convenience entries for C++ hosts.
//
// Replaces the CUDA-typed declarations of the reference's include/fesom2-accelerate.h:155-209
// (fct_ale_a1_accelerated, fct_ale_a2_accelerated, fct_ale_a1_a2_accelerated; implemented at
// src/fesom2-accelerate.cu:42-112 on the kernels kernels/fct_ale_a1.cu and fct_ale_a2.cu).  Same
// names, argument order, defaults and C linkage; the stream is a hipStream_t instead of a
// cudaStream_t, and `struct gpuMemory *` is the opaque handle that alloc_var_, reserve_var_ and
// transfer_mesh_ store in their `void **ret` (cast it: `(gpuMemory *)h`).
//
// Semantics (the reference kernels', which differ from src/reference.cpp's CPU a1/a2): every array
// has the single column stride maxLevels; a1 covers levels z < nLevels_nod2D(n) of nodes n < nNodes
// with fmax/fmin; a2 writes, per element e < nElements, UV_rhs(z, e) = (max, min) over its three
// nodes for z < nLevels_elem(e) - 1 and (-1e3, +1e3) for nLevels_elem(e) - 1 <= z < maxLevels - 1.
// Transfers: the inputs go host -> device before the kernels and the outputs device -> host after
// them, synchronously or on `stream` (asynchronous: await the stream before reading the host
// arrays).  The reference launches its kernels on the null stream; here they run on `stream`.
// Errors: no status argument (the reference has none); a failure is reported on stderr and in
// fesom2_last_error(), and nothing is launched.
#pragma once
#include <hip/hip_runtime_api.h>

#include "fesom2-accelerate.h"

struct gpuMemory;

extern "C" {
void fct_ale_a1_accelerated(const int maxLevels, const int nNodes, struct gpuMemory *nLevels_nod2D,
                            struct gpuMemory *fct_ttf_max, struct gpuMemory *fct_ttf_min,
                            struct gpuMemory *fct_low_order, struct gpuMemory *ttf, bool synchronous = true,
                            hipStream_t stream = nullptr);
void fct_ale_a2_accelerated(const int maxLevels, const int nElements, struct gpuMemory *nLevels_elem,
                            struct gpuMemory *elementNodes, struct gpuMemory *UV_rhs,
                            struct gpuMemory *fct_ttf_max, struct gpuMemory *fct_ttf_min, bool synchronous = true,
                            hipStream_t stream = nullptr);
void fct_ale_a1_a2_accelerated(const int maxLevels, const int nNodes, const int nElements,
                               struct gpuMemory *nLevels_nod2D, struct gpuMemory *nLevels_elem,
                               struct gpuMemory *elementNodes, struct gpuMemory *fct_ttf_max,
                               struct gpuMemory *fct_ttf_min, struct gpuMemory *fct_low_order,
                               struct gpuMemory *ttf, struct gpuMemory *UV_rhs, bool synchronous = true,
                               hipStream_t stream = nullptr);
}
