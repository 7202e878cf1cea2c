/*
 * fesom2-accelerate.h -- C-ABI of the MI355X-native FCT-ALE engine (libfesom2-accelerate.so).
 *
 * Drop-in for the reference's include/fesom2-accelerate.h:128-236 (ESiWACE-S1/fesom2-accelerate).
 * Every entry point keeps the reference's name, gfortran-style trailing underscore, by-pointer
 * arguments and meaning; device buffers are opaque handles passed as void** (the caller stores the
 * void* the library returned).  No CUDA/HIP or C++ types appear in any signature.
 *
 * Conventions (reference src/fesom2-accelerate.cu):
 *   istat      0 ok, 1 failure (message on stderr)
 *   alg_state  last completed step, for the caller's CPU fallback: pre_comm -> 6,
 *              inter_comm -> 7, post_comm -> 8 (reference :337, :354, :377); new c-step -> 9.
 *              vlimit 2/3 are computed on the GPU as well (the reference GPU path ignores vlimit).
 *   layouts    Fortran column-major: node fields (nl-1, nodes), fct_adf_v/area/area_inv (nl, nodes),
 *              fct_adf_h (nl-1, edges), UV_rhs (2, nl-1, elem); connectivity int32, 1-based.
 *   threading  one host thread per rank; all phase work is enqueued on *s; the caller awaits it
 *              with await_stream_ before touching host outputs.
 */
#ifndef FESOM2_ACCELERATE_H
#define FESOM2_ACCELERATE_H

#ifndef __cplusplus
#include <stdbool.h>
#endif

typedef double real_type; /* reference .h:10 */

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- memory / stream / device */

/* reference .h:146, impl src/fesom2-accelerate.cu:206-228: device = (rank % total_ranks) % ndev */
void set_mpi_rank_(int *rank, int *total_ranks);
/* reference .h:147, impl :114-127: allocate + synchronous upload of an int32 array of *size items */
void transfer_mesh_(void **ret, int *host_ptr, int *size, int *istat);
/* reference .h:148, impl :129-134: allocate *size doubles bound to host_ptr (no copy) */
void alloc_var_(void **ret, real_type *host_ptr, int *size, bool *create_event, int *istat);
/* reference .h:149, impl :136-141: device-only scratch of *size doubles */
void reserve_var_(void **ret, int *size, bool *create_event, int *istat);
/* reference .h:150, impl :143-154: pinned host doubles; istat 1 = fell back to malloc */
void allocate_pinned_doubles_(void **hostptr, int *size, int *istat);
/* reference .h:151, impl :156-161: rebind host pointer, synchronous H2D */
void transfer_var_(void **mem, real_type *host_ptr);
/* reference .h:152, impl :163-168: rebind host pointer, async H2D on *stream, optional event record */
void transfer_var_async_(void **mem, real_type *host_ptr, void **stream, bool *record_event);
/* reference .h:153, impl :170-186: heap stream handle; istat 1 = fell back to the null stream */
void make_stream_(void **stream, int *istat);
/* reference .h:154, impl :188-198 */
void await_stream_(void **s, int *istat);

/* ---------------------------------------------------------------- FCT-ALE phases (GPU) */

/* reference .h:156, impl :258-340: a1, a2, a3(+b1-vertical), b1-horizontal, b2; D2H fct_plus/minus */
void fct_ale_pre_comm_acc_(int *alg_state, void **s, void **fct_ttf_max, void **fct_ttf_min,
                           void **fct_plus, void **fct_minus, void **ttf, void **fct_LO,
                           void **fct_adf_v, void **fct_adf_h, void **UV_rhs, void **area_inv,
                           int *myDim_nod2D, int *eDim_nod2D, int *myDim_elem2D, int *myDim_edge2D,
                           int *nl, void **nlevels_nod2D, void **nlevels_elem2D, void **elem2D_nodes,
                           void **nod_in_elem2D_num, void **nod_in_elem2D, int *nod_in_elem2D_dim,
                           void **nod2D_edges, void **elem2D_edges, int *vlimit, real_type *flux_eps,
                           real_type *bignumber, real_type *dt);
/* reference .h:157, impl :342-356: b3-vertical on owned nodes; D2H fct_adf_v */
void fct_ale_inter_comm_acc_(int *alg_state, void **s, void **fct_plus, void **fct_minus,
                             void **fct_adf_v, int *myDim_nod2D, int *nl, void **nlevels_nod2D);
/* reference .h:158, impl :358-379: H2D fct_plus/minus (halo filled by the caller's exchange),
 * b3-horizontal on local edges; D2H fct_adf_h.  The 8th argument holds nlevels(elem): the
 * reference header names it nlevels_nod2D but its definition (:358) uses nlevels_elem2D. */
void fct_ale_post_comm_acc_(int *alg_state, void **s, void **fct_plus, void **fct_minus,
                            void **fct_adf_h, int *myDim_edge2D, int *nl, void **nlevels_elem2D,
                            int *nod_in_elem2D_dim, void **nod2D_edges, void **elem2D_edges);

/* ---------------------------------------------------------------- reference CPU-named entries
 * reference .h:142, :225, :229, :232, :235 (src/reference.cpp:289-438).  Same names and meaning on
 * host arrays; here they are executed by the GPU engine (stage, launch, copy back, synchronous). */
void fct_ale_a1_reference_(int *nNodes, int *nLevels_nod2D, int *nl, real_type *fct_ttf_max,
                           real_type *fct_ttf_min, real_type *fct_low_order, real_type *ttf);
void fct_ale_a2_reference_(int *nElements, int *nLevels_elem2D, int *nl, real_type *UV_rhs,
                           int *elem2D_nodes, real_type *fct_ttf_max, real_type *fct_ttf_min,
                           real_type *bignumber);
void fct_ale_a3_reference_(int *nNodes2D, int *nLevels_nod2D, int *nl, real_type *fct_ttf_max,
                           real_type *fct_ttf_min, real_type *fct_LO, real_type *UV_rhs,
                           real_type *fct_plus, real_type *fct_minus, real_type *fct_adf_v,
                           int *nod_in_elem2D, int *nod_in_elem2D_num, int *nod_in_elem2D_dim);
void fct_ale_a4_reference_(int *nNodes2D, int *nLevels_nod2D, int *nLevels_elem2D, int *nl,
                           int *nEdges2D, real_type *fct_plus, real_type *fct_minus,
                           real_type *fct_adf_h, real_type *area_inv, real_type *fct_ttf_max,
                           real_type *fct_ttf_min, int *edges, int *edge_tri, real_type *flux_eps,
                           real_type *dt);
void fct_ale_pre_comm_(int *alg_state, real_type *fct_ttf_max, real_type *fct_ttf_min,
                       real_type *fct_plus, real_type *fct_minus, real_type *ttf, real_type *fct_LO,
                       real_type *fct_adf_v, real_type *fct_adf_h, real_type *UV_rhs,
                       real_type *area_inv, int *myDim_nod2D, int *eDim_nod2D, int *myDim_elem2D,
                       int *myDim_edge2D, int *nl, int *nlevels_nod2D, int *nlevels_elem2D,
                       int *elem2D_nodes, int *nod_in_elem2D_num, int *nod_in_elem2D,
                       int *nod_in_elem2D_dim, int *nod2D_edges, int *elem2D_edges, int *vlimit,
                       real_type *flux_eps, real_type *bignumber, real_type *dt);

/* ================================================================ additions (not in the reference)
 * Everything below is new API; none of it changes the entry points above. */

/* c-step (docs/refactoring.md:292-314; reference kernels built but never launched):
 * c-vertical on owned nodes + c-horizontal gathered per owned node; alg_state -> 9. */
void fct_ale_c_acc_(int *alg_state, void **s, void **del_ttf_advvert, void **del_ttf_advhoriz,
                    void **ttf, void **fct_LO, void **hnode, void **hnode_new, void **fct_adf_v,
                    void **fct_adf_h, void **area, int *myDim_nod2D, int *eDim_nod2D,
                    int *myDim_edge2D, int *nl, void **nlevels_nod2D, void **nlevels_elem2D,
                    void **nod2D_edges, void **elem2D_edges, real_type *dt);

/* Fast mode (fesom2_set_path_(2)) only: bind the c-step's vertical fields to a tracer's fct_adf_v
 * once, so that fct_ale_pre_comm_acc_ -- which receives none of them -- also does c-vertical while
 * its plus/minus, raw fct_adf_v, ttf and fct_LO are in registers; fct_ale_c_acc_ then does
 * c-horizontal only.  The handles must be the ones later passed to fct_ale_c_acc_ (checked there),
 * and del_ttf_advvert must hold its pre-c-step value when pre_comm runs (FESOM2 fills it before
 * fct_ale).  Same results.  Null handles (all four) unbind.  istat 1 on invalid handles/sizes. */
void fesom2_bind_c_vertical_(int *istat, void **fct_adf_v, void **del_ttf_advvert, void **hnode,
                             void **hnode_new, void **area);

/* Fused phase 2 = b3-vertical + b3-horizontal + c-vertical + c-horizontal in one node-centric pass
 * (needs fct_plus/minus valid on the halo).  Same results as inter_comm + post_comm + c; alg_state -> 9. */
void fct_ale_post_comm_c_acc_(int *alg_state, void **s, void **fct_plus, void **fct_minus,
                              void **fct_adf_v, void **fct_adf_h, void **del_ttf_advvert,
                              void **del_ttf_advhoriz, void **ttf, void **fct_LO, void **hnode,
                              void **hnode_new, void **area, int *myDim_nod2D, int *eDim_nod2D,
                              int *myDim_edge2D, int *nl, void **nlevels_nod2D,
                              void **nlevels_elem2D, void **nod2D_edges, void **elem2D_edges,
                              real_type *dt);

/* alloc_var_ / reserve_var_ with 64-bit element counts (a 9.6M-node x 80-level mesh on one GPU has
 * 2.3e9-element fct_adf_h; the reference's int size stops at 2^31-1, and a negative int size is
 * rejected with istat = 1). */
void fesom2_alloc_var_i8_(void **ret, real_type *host_ptr, long long *size, bool *create_event, int *istat);
void fesom2_reserve_var_i8_(void **ret, long long *size, bool *create_event, int *istat);

/* Transfer mode.  0 (default) = reference semantics: pre_comm uploads fct_LO and downloads
 * fct_plus/minus, inter_comm downloads fct_adf_v, post_comm uploads fct_plus/minus and downloads
 * fct_adf_h, c downloads del_ttf_*.  1 = device resident: no implicit host transfers. */
void fesom2_set_resident_(int *resident);
/* Kernel path.  0 (default) = fused node-centric kernels; 1 = one kernel per reference step
 * (materialises fct_ttf_max/min and UV_rhs, honours FESOM2_NUM_KERNELS for bisection); 2 = the
 * reference entry sequence's fast mode: fct_ale_pre_comm_acc_ also does b3-vertical (the node's own
 * plus/minus are final after b2) and the block-internal edges' b3-horizontal, fct_ale_inter_comm_acc_
 * then only moves fct_adf_v, fct_ale_post_comm_acc_ limits the remaining edges.  Same results;
 * phase-2 entries other than inter_comm/post_comm refuse fct_adf_v/fct_adf_h touched this way. */
void fesom2_set_path_(int *path);
/* Build the derived mesh structures (edge/ring CSR, processing order) ahead of the first pass
 * (otherwise built lazily, synchronously, on first use).  Calls with ntracers > 1 run on a plan of
 * their own (smaller patches and blocks for the batch's tile order), built on the first such call
 * or by fesom2_mesh_info_ with *ninfo >= 10. */
void fesom2_prepare_mesh_(int *istat, int *myDim_nod2D, int *eDim_nod2D, int *myDim_elem2D,
                          int *myDim_edge2D, int *nl, void **nlevels_nod2D, void **nlevels_elem2D,
                          void **elem2D_nodes, void **nod_in_elem2D_num, void **nod_in_elem2D,
                          int *nod_in_elem2D_dim, void **nod2D_edges, void **elem2D_edges);
/* Diagnostics of the phase-1 mesh plan (built if needed): info[0] p1v block columns of the
 * block-internal edge lists (0 = none), [1] interior edges, [2] interior edges crossing p1v blocks,
 * [3] block-internal edges (limited inside fct_ale_pre_comm_v_acc_), [4] their edge cells;
 * [5, 10) the same for the plan of batched calls (ntracers > 1); [10], [11] the single-tracer plan's
 * cluster unions (p1v block columns, 0 = none; the largest union), [12], [13] the batched plan's.
 * *ninfo: capacity in (at most 14 used), entries written out. */
void fesom2_mesh_info_(int *istat, int *myDim_nod2D, int *eDim_nod2D, int *myDim_elem2D, int *myDim_edge2D,
                       int *nl, void **nlevels_nod2D, void **nlevels_elem2D, void **elem2D_nodes,
                       void **nod_in_elem2D_num, void **nod_in_elem2D, int *nod_in_elem2D_dim,
                       void **nod2D_edges, void **elem2D_edges, long long *info, int *ninfo);
/* The Infinity-Cache pass order the split, fused and reference-sequence entries use for a call of
 * *ntracers tracers on this mesh (mesh plan built if needed): *order bits 1 phase 1 and 4 the
 * c-step's node kernel walk their tile ranges backwards, 8 b3h stores the limited fluxes
 * cache-allocating; 0 = every kernel forwards with non-temporal flux stores.  On when the call's
 * fct_adf_h (ntracers x myDim_edge2D x (nl-1) doubles) is at most 192 MiB, or as the plan option
 * FESOM2_CACHE_ORDER forces.  Results never depend on it. */
void fesom2_pass_order_(int *istat, int *myDim_nod2D, int *eDim_nod2D, int *myDim_edge2D, int *nl,
                        void **nlevels_nod2D, void **nlevels_elem2D, void **nod2D_edges, void **elem2D_edges,
                        int *ntracers, int *order);
/* Copy a handle's device contents to/from a host array (no rebinding), synchronous. */
void fesom2_download_(void **mem, void *host_ptr, int *istat);
void fesom2_upload_(void **mem, void *host_ptr, int *istat);
/* Asynchronous device -> host copy of a handle on *stream: the mirror of transfer_var_async_ and
 * of the reference's asynchronous transfer_back (src/fesom2-accelerate.cu:230-253, which only the
 * phase entries call).  Rebinds the handle's host pointer to host_ptr (as transfer_var_async_
 * does) and enqueues the copy; the host awaits the stream (await_stream_) before reading it.
 * For a device-resident host (fesom2_set_resident_(1)) that uploads the producer's fields itself
 * and takes back only what it needs (e.g. del_ttf_advvert / del_ttf_advhoriz after the c-step).
 * istat 0 = ok. */
void fesom2_transfer_back_async_(void **mem, real_type *host_ptr, void **stream, int *istat);
/* Release a handle / stream / pinned buffer (the reference never frees). */
void fesom2_free_(void **mem);
void fesom2_free_stream_(void **stream);
/* hipGraph capture of everything the entry points enqueue on *s between begin and end (device-
 * resident mode; the meshes' plans must exist: run the sequence once or fesom2_prepare_mesh_ first;
 * one open capture per thread, ended on the stream it began on).  launch replays it on *s without
 * host-side work; free releases it.  istat 0 = ok.
 * A replay reuses what the calls read at capture time (handles, sizes, dt, flux_eps, bignumber,
 * vlimit, ntracers, path/FESOM2_* choices) and does not update alg_state.  Before each replay the
 * launch stream waits for the events of the buffers the captured calls wait on (transfer_var_async_
 * uploads with record_event, reference :293/:316/:326).  launch fails (istat 1) if a buffer, halo
 * plan or communicator the capture used has been freed since.  While any capture is open, calls
 * that would build a new mesh plan fail. */
void fesom2_graph_begin_(int *istat, void **s);
void fesom2_graph_end_(int *istat, void **s, void **graph);
void fesom2_graph_launch_(int *istat, void **graph, void **s);
void fesom2_graph_free_(void **graph);
/* Objects a graph's replays check (*n_uses) and buffer events they wait on (*n_waits); -1 = invalid. */
void fesom2_graph_info_(void **graph, int *n_uses, int *n_waits);
void fesom2_free_pinned_(void **hostptr);
/* Device-wide synchronisation and last error string (empty if none). */
void fesom2_device_sync_(int *istat);
const char *fesom2_last_error(void);
/* Per-kernel timing: while enabled, every launch is bracketed by HIP events on its stream.
 * Switching it on or off does not synchronise (the events are resolved when the statistics are read
 * or reset), so a harness may time a sample of the steps.  fesom2_kernel_stats_ writes "name count
 * total_ms" lines (NUL-terminated, truncated to *len bytes) and sets *len to the size needed. */
void fesom2_kernel_timing_(int *on);
/* Restrict the timing to launches named `name` (NULL or "": every launch).  Each timed launch adds
 * two events on its stream; timing one kernel keeps the others' boundaries free of them. */
void fesom2_kernel_timing_only_(const char *name);
void fesom2_kernel_timing_reset_(void);
void fesom2_kernel_stats_(char *buf, int *len);
/* Timing: create/record/elapsed on a stream (HIP events); used by the benchmark harness. */
void fesom2_event_create_(void **ev, int *istat);
void fesom2_event_record_(void **ev, void **s);
void fesom2_event_elapsed_(void **ev0, void **ev1, float *ms);
void fesom2_event_free_(void **ev);

/* ---------------------------------------------------------------- multi-GPU halo (RCCL over xGMI)
 * The reference leaves exchange_nod(fct_plus, fct_minus) to the Fortran host's MPI between
 * pre_comm and post_comm (docs/refactoring.md:199-200, :235).  This device-resident replacement
 * packs the owned columns neighbours need, exchanges them with grouped ncclSend/ncclRecv on a
 * communication stream and unpacks them into the halo columns. */
void fesom2_comm_unique_id_(char *id128, int *istat);
void fesom2_comm_init_(void **comm, char *id128, int *rank, int *nranks, int *istat);
void fesom2_comm_free_(void **comm);
/* What the communicator itself reports (ncclCommCount / ncclCommUserRank / ncclCommCuDevice):
 * lets a host (and bench.py) confirm how many ranks the RCCL exchange actually spans. */
void fesom2_comm_info_(void **comm, int *rank, int *nranks, int *device, int *istat);
/* Halo plan: per neighbour rank, the 1-based local node numbers to send (owned) and to receive
 * (halo), concatenated in neighbour order. */
void fesom2_halo_plan_(void **plan, int *nneigh, int *neigh_ranks, int *send_counts,
                       int *send_nodes, int *recv_counts, int *recv_nodes, int *nl, int *istat);
void fesom2_halo_plan_free_(void **plan);
/* Exchange fct_plus/fct_minus halo columns; enqueued on *s (work after it on *s sees the halo). */
void fct_ale_exchange_acc_(int *istat, void **s, void **comm, void **plan, void **fct_plus,
                           void **fct_minus);
/* Exchange + fused phase 2 with overlap: the exchange runs on the halo plan's communication stream
 * while b3h/b3v/cv/ch process the interior (no halo endpoint), the boundary follows once the halo
 * has arrived (docs/refactoring.md:199-235 ordering).  Same results as fct_ale_exchange_acc_ then
 * fct_ale_post_comm_c_acc_; alg_state -> 9. */
void fct_ale_exchange_post_comm_c_acc_(int *alg_state, void **s, void **comm, void **halo_plan,
                                       void **fct_plus, void **fct_minus, void **fct_adf_v,
                                       void **fct_adf_h, void **del_ttf_advvert,
                                       void **del_ttf_advhoriz, void **ttf, void **fct_LO,
                                       void **hnode, void **hnode_new, void **area,
                                       int *myDim_nod2D, int *eDim_nod2D, int *myDim_edge2D, int *nl,
                                       void **nlevels_nod2D, void **nlevels_elem2D,
                                       void **nod2D_edges, void **elem2D_edges, real_type *dt);

/* ---- multi-tracer batched variant (SURVEY.md 8(b) "new exports": several tracers per launch).
 * Per-tracer handles hold ntracers tracers one after another: ttf, fct_LO, fct_plus, fct_minus,
 * del_ttf_advvert, del_ttf_advhoriz (myDim_nod2D+eDim_nod2D)*(nl-1) doubles apart, fct_adf_v
 * (myDim_nod2D+eDim_nod2D)*nl apart, fct_adf_h myDim_edge2D*(nl-1) apart -- i.e. Fortran arrays
 * (nl-1, nod, ntracers), (nl, nod, ntracers), (nl-1, edge, ntracers).  Mesh fields (area,
 * area_inv, hnode, hnode_new) are shared.  Each tracer's results equal a single-tracer pass on
 * its slice.  Fused path only. */
void fct_ale_pre_comm_batched_acc_(int *alg_state, void **s, int *ntracers, void **fct_plus,
                                   void **fct_minus, void **ttf, void **fct_LO, void **fct_adf_v,
                                   void **fct_adf_h, void **area_inv, int *myDim_nod2D,
                                   int *eDim_nod2D, int *myDim_elem2D, int *myDim_edge2D, int *nl,
                                   void **nlevels_nod2D, void **nlevels_elem2D, void **elem2D_nodes,
                                   void **nod_in_elem2D_num, void **nod_in_elem2D,
                                   int *nod_in_elem2D_dim, void **nod2D_edges, void **elem2D_edges,
                                   int *vlimit, real_type *flux_eps, real_type *bignumber,
                                   real_type *dt);
void fct_ale_post_comm_c_batched_acc_(int *alg_state, void **s, int *ntracers, void **fct_plus,
                                      void **fct_minus, void **fct_adf_v, void **fct_adf_h,
                                      void **del_ttf_advvert, void **del_ttf_advhoriz, void **ttf,
                                      void **fct_LO, void **hnode, void **hnode_new, void **area,
                                      int *myDim_nod2D, int *eDim_nod2D, int *myDim_edge2D, int *nl,
                                      void **nlevels_nod2D, void **nlevels_elem2D,
                                      void **nod2D_edges, void **elem2D_edges, real_type *dt);
/* nod_columns = myDim_nod2D + eDim_nod2D (the per-tracer stride in columns). */
void fct_ale_exchange_batched_acc_(int *istat, void **s, void **comm, void **plan, int *ntracers,
                                   int *nod_columns, void **fct_plus, void **fct_minus);
/* FESOM's exchange_nod(a) / exchange_nod(a, b) on the device for (nl-1, nod) fields -- ttf and
 * fct_LO before phase 1, del_ttf_* after the c-step, fct_LO between iter_yn iterations
 * (SURVEY.md 8(f) 3).  *field_b may be NULL (one field); ntracers blocks nod_columns*(nl-1) apart. */
void fesom2_exchange_nod_acc_(int *istat, void **s, void **comm, void **plan, int *ntracers,
                             int *nod_columns, void **field_a, void **field_b);
void fct_ale_exchange_post_comm_c_batched_acc_(int *alg_state, void **s, void **comm, void **halo_plan,
                                               int *ntracers, void **fct_plus, void **fct_minus,
                                               void **fct_adf_v, void **fct_adf_h, void **del_ttf_advvert,
                                               void **del_ttf_advhoriz, void **ttf, void **fct_LO,
                                               void **hnode, void **hnode_new, void **area,
                                               int *myDim_nod2D, int *eDim_nod2D, int *myDim_edge2D,
                                               int *nl, void **nlevels_nod2D, void **nlevels_elem2D,
                                               void **nod2D_edges, void **elem2D_edges, real_type *dt);

/* ---- split by direction (the fastest pass): the vertical half of phase 2 (b3-vertical, c-vertical)
 * reads only the node's own column, so it runs inside phase 1; phase 2 keeps b3-horizontal and
 * c-horizontal.  Same results as pre_comm + post_comm_c.  ntracers as the batched entries (1 = the
 * single-tracer layouts; fct_adf_v, del_ttf_advvert then sized like fct_ale_post_comm_c_acc_). */
/* a1..b2 + b3v + cv: fct_plus/minus, limited fct_adf_v, del_ttf_advvert updated.  alg_state -> 7. */
void fct_ale_pre_comm_v_acc_(int *alg_state, void **s, int *ntracers, void **fct_plus, void **fct_minus,
                             void **ttf, void **fct_LO, void **fct_adf_v, void **fct_adf_h, void **area_inv,
                             void **area, void **hnode, void **hnode_new, void **del_ttf_advvert,
                             int *myDim_nod2D, int *eDim_nod2D, int *myDim_elem2D, int *myDim_edge2D, int *nl,
                             void **nlevels_nod2D, void **nlevels_elem2D, void **elem2D_nodes,
                             void **nod_in_elem2D_num, void **nod_in_elem2D, int *nod_in_elem2D_dim,
                             void **nod2D_edges, void **elem2D_edges, int *vlimit, real_type *flux_eps,
                             real_type *bignumber, real_type *dt);
/* [halo exchange of fct_plus/minus overlapped with the interior, when *comm and *halo_plan are
 * set] + b3h + c-horizontal.  alg_state -> 9. */
void fct_ale_post_comm_h_acc_(int *alg_state, void **s, int *ntracers, void **comm, void **halo_plan,
                              void **fct_plus, void **fct_minus, void **fct_adf_h, void **del_ttf_advhoriz,
                              void **area, int *myDim_nod2D, int *eDim_nod2D, int *myDim_edge2D, int *nl,
                              void **nlevels_nod2D, void **nlevels_elem2D, void **nod2D_edges,
                              void **elem2D_edges, real_type *dt);

/* ---- iter_yn iterative FCT (docs/refactoring.md:227-229, :258-260, :265-290).
 * Phase 2 of a non-final iteration, after the exchange of fct_plus/minus: b3 limiting with the
 * remainders fct_adf_v2 = (1-ae) fct_adf_v (levels 2..nlevels-1) and fct_adf_h2 = (1-ae) fct_adf_h,
 * fct_LO += the limited flux divergence / hnode_new (owned nodes; halo entries of fct_LO are left
 * alone -- the caller's LO halo exchange refreshes them), then fct_adf_v <- fct_adf_v2 and
 * fct_adf_h <- fct_adf_h2.  No c-step; the caller runs fct_ale again.  alg_state -> 9. */
void fct_ale_post_comm_iter_acc_(int *alg_state, void **s, void **fct_plus, void **fct_minus,
                                 void **fct_adf_v, void **fct_adf_h, void **fct_adf_v2,
                                 void **fct_adf_h2, void **fct_LO, void **hnode_new, void **area,
                                 int *myDim_nod2D, int *eDim_nod2D, int *myDim_edge2D, int *nl,
                                 void **nlevels_nod2D, void **nlevels_elem2D, void **nod2D_edges,
                                 void **elem2D_edges, real_type *dt);
void fct_ale_post_comm_iter_batched_acc_(int *alg_state, void **s, int *ntracers, void **fct_plus,
                                         void **fct_minus, void **fct_adf_v, void **fct_adf_h,
                                         void **fct_adf_v2, void **fct_adf_h2, void **fct_LO,
                                         void **hnode_new, void **area, int *myDim_nod2D,
                                         int *eDim_nod2D, int *myDim_edge2D, int *nl,
                                         void **nlevels_nod2D, void **nlevels_elem2D,
                                         void **nod2D_edges, void **elem2D_edges, real_type *dt);

#ifdef __cplusplus
}
#endif
#endif /* FESOM2_ACCELERATE_H */
