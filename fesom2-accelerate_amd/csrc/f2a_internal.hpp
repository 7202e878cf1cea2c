// f2a_internal.hpp -- internal types shared by the host orchestration and the HIP kernels.
//
// Not part of the public C-ABI (that is include/fesom2-accelerate.h).
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>
#include <cstdlib>

// The tuning build (make tuning -> lib/libfesom2-accelerate-tuning.so, F2A_TUNING=1) reads the
// FESOM2_* A/B knobs tools/sweep_env.sh sweeps (other gather batches, wave counts, cache policies,
// tile orders, timing-only ablations).  The product library compiles every knob to its measured default:
// no environment variable changes its kernel selection (the plan options of get_plan aside,
// which are read once when a mesh plan is built; INTEGRATION.md lists them).
#ifndef F2A_TUNING
#define F2A_TUNING 0
#endif

namespace f2a {

// A/B knob: the environment in the tuning build, the default in the product library.
static inline int knob(const char *name, int dflt)
{
#if F2A_TUNING
    const char *e = getenv(name);
    return e ? atoi(e) : dflt;
#else
    (void)name;
    return dflt;
#endif
}

using real = double;

// Slack behind every device array the library allocates (Buffer): kernels read odd-L columns in
// 16-byte level pairs without shifting the last pair, so the last column of an array reads 8 bytes
// past its end (see ldo in f2a_device.hpp).
constexpr size_t kAllocPad = 64;

// Buffer handle returned through void** (replaces the reference's struct gpuMemory,
// include/fesom2-accelerate.h:19-28).  `magic` lets every entry point reject a stale or foreign
// handle loudly instead of dereferencing it.
struct Buffer {
    static constexpr uint32_t kMagic = 0xF2A0B0F1u;
    uint32_t magic = kMagic;
    void *host_pointer = nullptr;
    void *device_pointer = nullptr;
    size_t size = 0;  // bytes
    // readable slack behind `size` (kAllocPad for every array allocate() makes): need() refuses a
    // buffer without it, so an entry that ever wraps a foreign device pointer (an OpenACC/OpenMP
    // array of the host) fails loudly instead of letting the odd-L pair loads read past its end
    size_t pad = 0;
    hipEvent_t event = nullptr;
    bool has_event = false;
    uint64_t serial = 0;  // live-object serial (track_object): graph replays check it is unchanged
    uint64_t version = 0;  // bumped by every host -> device upload through the library (h2d, fesom2_upload_)
    // phase mark (f2a_host.hpp): on fct_adf_h the mesh plan whose block-internal edges a p1v launch
    // limited (the phase-2 entry then limits the others), on fct_adf_v the plan whose phase-1 launch
    // did b3-vertical; cleared by the entry that finishes the phase and by every upload
    const void *int_plan = nullptr;
    uint64_t int_serial = 0;
    // fct_adf_v only: the c-step's vertical fields bound by fesom2_bind_c_vertical_ (owned)
    struct CvBinding *cv = nullptr;
};

// fesom2_bind_c_vertical_: del_ttf_advvert, hnode, hnode_new, area with their live serials
struct CvBinding {
    Buffer *b[4];
    uint64_t serial[4];
};

// One incident edge of a node in the node->edge CSR (ascending edge order per node, which is the
// order in which the reference's edge loops touch the node: reference.cpp:406-425).
struct EdgeRef {
    int edge;   // 0-based local edge
    int code;   // (lev << 1) | second: lev = max(nl1, nl2) levels the edge carries
                // (reference.cpp:412-414); second = this node is edges(2,e)
    int other;  // 0-based local node at the other end (owned if < myDim_nod2D)
};

// One node of a node's cluster (the union of the nodes of its adjacent elements).  `lev` is the
// number of levels on which the node takes part in the cluster bound:
// max over adjacent elements e that contain it of (nlevels(e) - 1)  (reference.cpp:331, :363-377).
// In the processing-order copies (MeshPlanDev::p_ring, NodeRec::ring) the node itself is the last
// entry of its slice, with lev = NodeInfo::self_lev: k_p1 reads its own column once for the
// cluster bound, b2 and the vertical tail, and gathers only [r0, r1 - 1).
struct RingRef {
    int node;
    int lev;
};

// One owned node at one position of the processing order (32 bytes, one load per cell).
// [r0, r1) / [e0, e1) index the processing-order copies of the cluster / edge CSRs.
struct NodeInfo {
    int n;     // 0-based local node
    int Ln;    // nlevels_nod2D(n) - 1
    int r0, r1;
    int e0, e1;
    int zdry;  // min over adjacent elements of (nlevels(e) - 1); levels >= zdry see the a2 fill
    int self_lev;  // levels on which the node itself is in its cluster (max over its elements)
};

// NodeInfo plus the first kRecRing cluster and kRecEdge edge entries inline (192 bytes, 16-byte
// aligned): a block loads its columns' records with one coalesced sweep into LDS, so the gathers
// depend on a single global load instead of NodeInfo -> CSR -> gather.  Entries beyond the inline
// capacity stay in the processing-order CSRs at [r0 + kRecRing, r1) / [e0 + kRecEdge, e1).
constexpr int kRecRing = 8, kRecEdge = 8;
constexpr int kB3hPackSlots = 640, kB3hPackEdges = 256;  // packed b3h block: level pairs, edges
struct alignas(16) NodeRec {
    NodeInfo info;
    RingRef ring[kRecRing];
    EdgeRef edge[kRecEdge];
};
static_assert(sizeof(NodeRec) == 192, "NodeRec layout");

// Device-side view of the derived mesh structures of one (mesh, partition) pair.
struct MeshPlanDev {
    int n_owned = 0;       // myDim_nod2D
    // block size of the column-group kernels: 2^gshift times group_columns' natural G (the batched
    // plan halves it, see get_plan), or exactly gcols columns when > 0
    int gshift = 0;
    int gcols = 0;
    int n_total = 0;       // myDim_nod2D + eDim_nod2D
    int n_edges = 0;       // myDim_edge2D
    int nl = 0;
    // node -> incident edges, owned nodes only
    const int *edge_ptr = nullptr;     // [n_owned + 1]
    const EdgeRef *edges = nullptr;    // [edge_ptr[n_owned]]
    // node -> cluster nodes, owned nodes only (needs elem2D_nodes / nod_in_elem2D)
    const int *ring_ptr = nullptr;     // [n_owned + 1]
    const RingRef *ring = nullptr;
    const int *zdry = nullptr;         // [n_owned] min over adjacent elements of (nlevels(e)-1)
    // locality-aware processing order (compact BFS patches of the node graph, see build_plan):
    // owned nodes and local edges in the order the fused kernels visit them, with the CSRs
    // re-laid out in that order
    const NodeInfo *node_info = nullptr;  // [n_owned]
    const NodeRec *node_rec = nullptr;    // [n_owned]
    const EdgeRef *p_edges = nullptr;     // node->edge CSR, processing order
    const RingRef *p_ring = nullptr;      // cluster CSR, processing order (if has ring)
    const int4 *p_edge_info = nullptr;    // [n_edges] {node1, node2, lev, edge}, processing order,
                                          // interior edges (both endpoints owned) first
    int n_edge_interior = 0;
    // packed b3h (variable depth): blocks of consecutive p_edge_info edges holding at most
    // kB3hPackSlots level pairs; b3p_desc[b] = {first edge, edges}, b3p_off[k] = slot offset of edge k
    // in its block; descriptors [0, b3p_nint) cover the interior edges, the rest the boundary ones
    const int2 *b3p_desc = nullptr;
    const unsigned short *b3p_off = nullptr;
    int b3p_nint = 0, b3p_ndesc = 0, b3p_cap = 0;  // b3p_cap: level pairs per block
    // the interior edges crossing p1v blocks (b3h's list on the split path when p1v limits the
    // block-internal ones), processing order, packed the same way
    int n_ext_interior = 0;
    const int4 *p_edge_ext = nullptr;
    const int2 *b3x_desc = nullptr;
    const unsigned short *b3x_off = nullptr;
    int b3x_ndesc = 0, b3x_cap = 0;
    int b3x_slots = 0;  // > 0: every crossing edge has this many level-pair slots (regular packing)
    int b3p_slots_int = 0, b3p_slots_bnd = 0;  // the same for b3p's interior / boundary edge ranges
    // b3-horizontal of the block-internal edges inside p1v (both endpoints' plus/minus are in the
    // block's LDS after b2): for p1v block b (int_G positions of the processing order) the entries
    // int_edges[int_ptr[b] .. int_ptr[b+1]) = {edge, column of edges(1,e), column of edges(2,e), lev}
    int int_G = 0;                        // 0: no internal-edge lists
    int int_max = 0;                      // most internal edges of one block
    // tuning build (FESOM2_P1V_STASH): the first endpoint's EdgeRef of each internal edge carries
    // (slot + 1) << kStashShift, slot = the edge's index in its block's list; p1v then keeps the
    // raw flux its b1h gather read in an LDS stash instead of re-reading it for the limiter
    int int_stash = 0;
    const int *int_ptr = nullptr;
    const int4 *int_edges = nullptr;
    // cluster union of each p1v block (the tuning build's FESOM2_P1V_UNION): block b's distinct
    // cluster nodes cu_node[cu_ptr[b] .. cu_ptr[b+1]), its own columns first (slot j = column j);
    // every processing-order RingRef then carries (slot + 1) << kStashShift above its level count,
    // and p1v stages the union's LO/ttf columns into LDS once per block (global -> LDS DMA) instead
    // of gathering each column's cluster separately
    int cu_G = 0;    // p1v columns per block the lists were built for (0: none)
    int cu_max = 0;  // most union nodes of one block
    const int *cu_ptr = nullptr;
    const int *cu_node = nullptr;
    // phase-2 node records: interior nodes (every incident edge interior) first, then boundary
    // nodes; interior work needs no halo values, so it can overlap the halo exchange
    const NodeRec *p2_rec = nullptr;      // [n_owned]
    int n_p2_interior = 0;
    int max_degree = 0;                   // most edges at one owned node
};

// Batched tracers: `n` tracers whose per-tracer arrays follow each other in one buffer, `node`
// elements apart for (L, nodes) fields, `lev` apart for (nl, nodes) fields (fct_adf_v), `edge` apart
// for fct_adf_h.  Mesh-only fields (area, area_inv, hnode, hnode_new) are shared.  Block tiles map
// to (column group, tracer) with the tracer fastest, so the n blocks of one column group run back to
// back on one XCD and share its L2 for the records and the shared fields.
struct Tracers {
    int n = 1;
    size_t node = 0, lev = 0, edge = 0;
    // pass order (pass_order, f2a_host.hpp): bit 0 the p1 kernels and bit 2 the p2 node kernels
    // walk each XCD's tile range backwards, bit 3 b3h stores the limited fluxes cache-allocating
    int order = 0;
};

// Kernel launchers (fct_ale_kernels.hip).  All enqueue on `s` and return hipGetLastError().
struct P1Args {
    int n_owned, nl, vlimit;
    const int *nlev_nod;
    const real *ttf, *LO, *adf_v, *adf_h, *area_inv;
    real *plus, *minus;
    real dt, eps, big;
    Tracers tr;
    // vertical part of phase 2 in the same kernel (launch_p1v: b3v + cv on the own column)
    const real *area = nullptr, *hnode = nullptr, *hnode_new = nullptr;
    real *del_v = nullptr;
};
hipError_t launch_p1_fused(const MeshPlanDev &mp, const P1Args &a, hipStream_t s);
// phase 1 + the vertical half of phase 2 (b3v, cv need only the node's own column: no halo), then
// phase 2's horizontal half alone (launch_p2h: c-horizontal; b3h stays its own kernel)
hipError_t launch_p1v(const MeshPlanDev &mp, const P1Args &a, hipStream_t s);
// phase 1 + b3v (+ the block-internal edges' b3h), no cv: fct_ale_pre_comm_acc_ in the reference
// sequence's fast mode (no area/hnode/hnode_new/del_v needed)
hipError_t launch_p1_b3v(const MeshPlanDev &mp, const P1Args &a, hipStream_t s);
// columns per p1v block for nl levels (the shape launch_p1v uses; the plan's int_G) at the plan's
// group shift, and its slots (threads) per column
int p1v_group_columns(int nl, int shift, int cols = 0);
int p1v_slots(int nl);
// launch_p1v limits the block-internal edges' fct_adf_h itself (b3h must then skip them)
bool p1v_limits_internal(const MeshPlanDev &mp, const P1Args &a);
constexpr int kMaxInternal = 64;  // most block-internal edges a p1v block limits (LDS staging)
constexpr int kStashShift = 12;   // EdgeRef::code bits above the level count (lev < 2048) and `second`
constexpr int kLevMask = 0x7FF;
// LDS of that staging (int4 entries + int slot offsets), rounded to whole doubles
__host__ __device__ constexpr size_t p1_internal_lds_bytes()
{
    return (kMaxInternal * sizeof(int4) + (kMaxInternal + 1) * sizeof(int) + 7) / 8 * 8;
}
// dynamic LDS of a phase-1 block (k_p1): tvert max/min, the G NodeRecs, the internal-edge staging,
// and for vlimit 2/3 the own columns' max(LO, ttf)
inline size_t p1_lds_bytes(int G, int L, int vlimit, bool internal)
{
    return (2 + (vlimit != 1 ? 1 : 0)) * (size_t)G * L * sizeof(double) + (size_t)G * 192 +
           (internal ? p1_internal_lds_bytes() : 0);
}
// the cluster-union staging behind `base` bytes of a p1v block's LDS (MeshPlanDev::cu_ptr): 16-byte
// aligned LO | ttf images of cu_max columns of 2S doubles (S level-pair slots), then the node ids
inline size_t p1_union_lds_bytes(size_t base, int cu_max, int S)
{
    return (base + 15) / 16 * 16 + 2 * (size_t)cu_max * 2 * S * sizeof(double) + (size_t)cu_max * sizeof(int);
}

struct P2Args {
    int nl;
    const NodeRec *nodes;   // processing positions to run (a subset of the plan's node_rec)
    int count;
    const real *plus, *minus, *ttf, *LO, *hnode, *hnode_new, *area;
    real *adf_v, *adf_h, *del_v, *del_h;
    real dt;
    Tracers tr;
};
hipError_t launch_p2_fused(const MeshPlanDev &mp, const P2Args &a, hipStream_t s);
hipError_t launch_p2h(const MeshPlanDev &mp, const P2Args &a, hipStream_t s);
// b3-horizontal over all local edges of the plan (edge groups, flat levels)
hipError_t launch_b3h_fused(const MeshPlanDev &mp, int nl, int begin, int count, const real *plus,
                            const real *minus, real *adf_h, const Tracers &tr, hipStream_t s);
// b3-horizontal over the interior edges crossing p1v blocks (mp.p_edge_ext)
hipError_t launch_b3h_ext(const MeshPlanDev &mp, int nl, const real *plus, const real *minus, real *adf_h,
                          const Tracers &tr, hipStream_t s);
// reference-sequence entries on the fused path: b3v and the c-step (cv + ch over the processing
// order) with the production kernels' column-group shape
hipError_t launch_b3v_cols(int n_owned, int nl, const int *nlev, const real *plus, const real *minus, real *adf_v,
                           hipStream_t s);
hipError_t launch_c_fused(const MeshPlanDev &mp, const P2Args &a, hipStream_t s);
// b3-horizontal over an explicit edge list ({node1, node2, lev, edge}, 0-based)
hipError_t launch_b3h_edges(const int4 *einfo, int count, int nl, const real *plus, const real *minus,
                            real *adf_h, const Tracers &tr, hipStream_t s);
// iter_yn phase 2 (docs/refactoring.md:227-229, :258-260, :265-290): node kernel = b3v writing
// fct_adf_v2, LO update from the limited vertical and horizontal fluxes (recomputed in-thread from
// plus/minus of both edge endpoints), then fct_adf_v <- fct_adf_v2 over the whole column; the
// edge kernel (after it) writes fct_adf_h2 = (1-ae) adf_h and fct_adf_h <- fct_adf_h2.
struct P2IterArgs {
    int nl;
    const NodeRec *nodes;
    int count;
    const int *edges;  // nod2D_edges (2, E), 1-based: the other endpoint of an edge
    const real *plus, *minus, *hnode_new, *area, *adf_h;
    real *LO, *adf_v, *adf_v2;
    real dt;
    Tracers tr;
};
hipError_t launch_p2_iter(const MeshPlanDev &mp, const P2IterArgs &a, hipStream_t s);
hipError_t launch_b3h_iter(const MeshPlanDev &mp, int nl, const real *plus, const real *minus, real *adf_h,
                           real *adf_h2, const Tracers &tr, hipStream_t s);
// columns per block for S slots per column (G*S fills whole wave64 iterations where possible),
// times 2^shift
int group_columns(int S, int shift = 0);

// Stepwise kernels, one per reference step.
hipError_t launch_a1(int n_nodes, int nl, const int *nlev_nod, const real *LO, const real *ttf,
                     real *tmax, real *tmin, hipStream_t s);
hipError_t launch_a2(int n_elem, int nl, const int *nlev_elem, const int *elem2D_nodes,
                     const real *tmax, const real *tmin, real *UV, real big, hipStream_t s);
hipError_t launch_a3(int n_owned, int nl, int vlimit, const int *nlev_nod, const int *nie,
                     const int *nie_num, int dim, const real *UV, const real *LO, real *tmax,
                     real *tmin, hipStream_t s);
hipError_t launch_b1v(int n_owned, int nl, const int *nlev_nod, const real *adf_v, real *plus,
                      real *minus, hipStream_t s);
hipError_t launch_b1h(const MeshPlanDev &mp, int nl, const real *adf_h, real *plus, real *minus,
                      hipStream_t s);
hipError_t launch_b2(int n_owned, int nl, const int *nlev_nod, const real *area_inv,
                     const real *tmax, const real *tmin, real *plus, real *minus, real dt,
                     real eps, hipStream_t s);
hipError_t launch_b3v(int n_owned, int nl, const int *nlev_nod, const real *plus,
                      const real *minus, real *adf_v, hipStream_t s);
hipError_t launch_b3h(int n_edges, int nl, const int *nlev_elem, const int *edges,
                      const int *edge_tri, const real *plus, const real *minus, real *adf_h,
                      hipStream_t s);
hipError_t launch_b3h_list(const int *edge_list, int count, int nl, const int *nlev_elem,
                           const int *edges, const int *edge_tri, const real *plus,
                           const real *minus, real *adf_h, hipStream_t s);
hipError_t launch_cv(int n_owned, int nl, const int *nlev_nod, const real *ttf, const real *hnode,
                     const real *LO, const real *hnode_new, const real *adf_v, const real *area,
                     real *del_v, real dt, hipStream_t s);
hipError_t launch_ch(const MeshPlanDev &mp, int nl, const real *adf_h, const real *area,
                     real *del_h, real dt, hipStream_t s);

// Halo pack / unpack of the columns of one or two (L, nodes) fields (`minus` may be null) of ntr
// tracers (`stride` elements apart); the buffer holds [list position][tracer][field L (| field L)],
// so each neighbour's part stays contiguous.
hipError_t launch_halo_pack(const int *nodes, int count, int L, int ntr, size_t stride, const real *plus,
                            const real *minus, real *buf, hipStream_t s);
hipError_t launch_halo_unpack(const int *nodes, int count, int L, int ntr, size_t stride, const real *buf,
                              real *plus, real *minus, hipStream_t s);

}  // namespace f2a
