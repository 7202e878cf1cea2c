/*
 * synth.c -- deterministic synthetic FESOM-like meshes and fields for benchmarks and tests.
 *
 * The reference ships no meshes; its tuning scripts draw unseeded random
 * connectivity (e.g. kernels/fct_ale_b1_horizontal.py:119-123).  This generator builds a periodic-x
 * structured triangulation with FESOM's array conventions instead (docs/refactoring.md:325-356):
 *
 *   nodes      id(i,j) = j*nx + i                         (row-major, spatially sorted)
 *   quads      q(i,j)  = j*nx + i,  j < ny-1             two triangles per quad:
 *              lower 2q   = [id(i,j), id(i+1,j), id(i+1,j+1)]
 *              upper 2q+1 = [id(i,j), id(i+1,j+1), id(i,j+1)]       (i+1 taken mod nx)
 *   edges      per row j, per column i: horizontal (i,j)-(i+1,j); if j < ny-1 also
 *              vertical (i,j)-(i,j+1) and diagonal (i,j)-(i+1,j+1)
 *   edge_tri   the two triangles of an edge, 1-based, second = 0 on the y boundary
 *   nod_in_elem2D(dim, N)  adjacent triangles per node, ascending, 1-based, zero padded
 *   nlevels(elem)          uniform in [3, nl] (parity meshes) or nl everywhere (full depth)
 *   nlevels_nod2D(n)       max over adjacent triangles (FESOM's definition)
 *
 * Every random value is a pure function of (seed, field, global index) through splitmix64, and
 * every distribution uses only exact IEEE operations, so a partition of the mesh regenerates the
 * same bits as the whole mesh on any machine.
 */
#include <stdint.h>
#include <string.h>
#include <math.h>

static inline uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static inline uint64_t hash3(uint64_t seed, uint64_t field, uint64_t index)
{
    return mix64(mix64(seed * 0x2545F4914F6CDD1Dull + field) ^ index);
}

static inline double unif(uint64_t h) { return (double)(h >> 11) * 0x1.0p-53; }

/* sizes of the nx x ny periodic-x triangulation */
void synth_mesh_sizes(int nx, int ny, int64_t *nodes, int64_t *elems, int64_t *edges, int *dim)
{
    *nodes = (int64_t)nx * ny;
    *elems = 2 * (int64_t)nx * (ny - 1);
    *edges = 3 * (int64_t)nx * (ny - 1) + nx;
    *dim = 6;
}

/*
 * Build connectivity.  Arrays (caller-allocated, int32, Fortran 1-based values):
 * elem2D_nodes[3T], edges[2E], edge_tri[2E], nie_num[N], nie[6N], nlev_elem[T], nlev_nod[N].
 * full_depth != 0 -> every element has nl levels.
 */
int synth_mesh_build(int nx, int ny, int nl, uint64_t seed, int full_depth, int *elem2D_nodes,
                     int *edges, int *edge_tri, int *nie_num, int *nie, int *nlev_elem,
                     int *nlev_nod)
{
    if (nx < 3 || ny < 2 || nl < 3)
        return 1;
    const int64_t N = (int64_t)nx * ny;
    const int64_t T = 2 * (int64_t)nx * (ny - 1);
#define ID(i, j) ((int64_t)(j) * nx + (((i) + nx) % nx))
#define QD(i, j) ((int64_t)(j) * nx + (((i) + nx) % nx))
    for (int j = 0; j < ny - 1; j++)
        for (int i = 0; i < nx; i++) {
            int64_t q = QD(i, j);
            int *lo = elem2D_nodes + 3 * (2 * q), *up = elem2D_nodes + 3 * (2 * q + 1);
            lo[0] = (int)ID(i, j) + 1;
            lo[1] = (int)ID(i + 1, j) + 1;
            lo[2] = (int)ID(i + 1, j + 1) + 1;
            up[0] = (int)ID(i, j) + 1;
            up[1] = (int)ID(i + 1, j + 1) + 1;
            up[2] = (int)ID(i, j + 1) + 1;
        }
    int64_t e = 0;
    for (int j = 0; j < ny; j++)
        for (int i = 0; i < nx; i++) {
            /* horizontal */
            edges[2 * e] = (int)ID(i, j) + 1;
            edges[2 * e + 1] = (int)ID(i + 1, j) + 1;
            if (j < ny - 1) {
                edge_tri[2 * e] = (int)(2 * QD(i, j)) + 1;                         /* lower above */
                edge_tri[2 * e + 1] = (j > 0) ? (int)(2 * QD(i, j - 1) + 1) + 1 : 0; /* upper below */
            } else {
                edge_tri[2 * e] = (int)(2 * QD(i, j - 1) + 1) + 1;
                edge_tri[2 * e + 1] = 0;
            }
            e++;
            if (j < ny - 1) {
                /* vertical */
                edges[2 * e] = (int)ID(i, j) + 1;
                edges[2 * e + 1] = (int)ID(i, j + 1) + 1;
                edge_tri[2 * e] = (int)(2 * QD(i, j) + 1) + 1;
                edge_tri[2 * e + 1] = (int)(2 * QD(i - 1, j)) + 1;
                e++;
                /* diagonal */
                edges[2 * e] = (int)ID(i, j) + 1;
                edges[2 * e + 1] = (int)ID(i + 1, j + 1) + 1;
                edge_tri[2 * e] = (int)(2 * QD(i, j)) + 1;
                edge_tri[2 * e + 1] = (int)(2 * QD(i, j) + 1) + 1;
                e++;
            }
        }
#undef ID
#undef QD
    for (int64_t t = 0; t < T; t++)
        nlev_elem[t] = full_depth ? nl : 3 + (int)(hash3(seed, 1, (uint64_t)t) % (uint64_t)(nl - 2));
    memset(nie_num, 0, sizeof(int) * N);
    memset(nie, 0, sizeof(int) * 6 * N);
    for (int64_t n = 0; n < N; n++)
        nlev_nod[n] = 0;
    /* ascending element order per node falls out of the ascending element loop */
    for (int64_t t = 0; t < T; t++)
        for (int k = 0; k < 3; k++) {
            int64_t n = elem2D_nodes[3 * t + k] - 1;
            int c = nie_num[n]++;
            nie[6 * n + c] = (int)t + 1;
            if (nlev_elem[t] > nlev_nod[n])
                nlev_nod[n] = nlev_elem[t];
        }
    return 0;
}

/*
 * Fill a column-major field out[c*stride + z], c < ncols, z < stride with values keyed on
 * (seed, field, gid[c]*stride + z); gid == NULL means gid[c] = c.
 * dist 0: uniform in [a, b);  dist 1: a + b*g, g ~ Irwin-Hall(4) scaled to unit variance.
 */
void synth_fill(uint64_t seed, int field, int dist, int64_t ncols, int stride, const int64_t *gid,
                double a, double b, double *out)
{
    const double s3 = 1.7320508075688772; /* sqrt(3) */
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < ncols; c++) {
        const uint64_t g = (uint64_t)(gid ? gid[c] : c) * (uint64_t)stride;
        double *o = out + c * (int64_t)stride;
        for (int z = 0; z < stride; z++) {
            uint64_t h = hash3(seed, (uint64_t)field, g + (uint64_t)z);
            if (dist == 0) {
                o[z] = a + (b - a) * unif(h);
            } else {
                double u = unif(h) + unif(mix64(h ^ 0x1ull)) + unif(mix64(h ^ 0x2ull)) +
                           unif(mix64(h ^ 0x3ull));
                o[z] = a + b * ((u - 2.0) * s3);
            }
        }
    }
}

/*
 * Levels of elements [t0, t0 + count) of the triangulation synth_mesh_build makes with the same
 * (nl, seed, full_depth): the strip generator of fesom2_amd/partition.py builds a rank's local mesh
 * from these without the global mesh.
 */
void synth_elem_levels(int nl, uint64_t seed, int full_depth, int64_t t0, int64_t count, int *out)
{
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < count; k++)
        out[k] = full_depth ? nl : 3 + (int)(hash3(seed, 1, (uint64_t)(t0 + k)) % (uint64_t)(nl - 2));
}
