/*
 * sanitize_check.c -- host-side sanitizer run of the test infrastructure (TEST ONLY).
 *
 * Builds synthetic meshes with csrc/synth.c, runs the oracle's full pass and its iter_yn branch
 * (oracle_b3v/b3h with fct_adf_*2, oracle_lo_update) on them, and exits 0.  Compiled with
 * -fsanitize=address,undefined by tests/test_sanitizers.py (sanitizers on host code;
 * GPU sanitizers are not available on this pool).  Every array is allocated at exactly the size
 * the ABI documents, so an out-of-bounds index in the restatement or the mesh generator trips ASan.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

void synth_mesh_sizes(int nx, int ny, int64_t *nodes, int64_t *elems, int64_t *edges, int *dim);
int synth_mesh_build(int nx, int ny, int nl, uint64_t seed, int full_depth, int *elem2D_nodes,
                     int *edges, int *edge_tri, int *nie_num, int *nie, int *nlev_elem, int *nlev_nod);
void synth_fill(uint64_t seed, int field, int dist, int64_t ncols, int stride, const int64_t *gid,
                double a, double b, double *out);
int oracle_full_pass(double *ttf_max, double *ttf_min, double *plus, double *minus,
                     const double *ttf, const double *LO, double *adf_v, double *adf_h,
                     double *UV_rhs, const double *area, const double *area_inv,
                     const double *hnode, const double *hnode_new, double *del_v, double *del_h,
                     int myDim_nod2D, int eDim_nod2D, int myDim_elem2D, int myDim_edge2D, int nl,
                     const int *nlev_nod, const int *nlev_elem, const int *elem2D_nodes,
                     const int *nie_num, const int *nie, int dim, const int *edges,
                     const int *edge_tri, int vlimit, double flux_eps, double big, double dt);
void oracle_b3v(int nNodes, const int *nlev_nod, int nl, double *adf_v, const double *plus,
                const double *minus, double *adf_v2);
void oracle_b3h(int nEdges, const int *nlev_elem, int nl, const int *edges, const int *edge_tri,
                double *adf_h, const double *plus, const double *minus, double *adf_h2);
void oracle_lo_update(int nNodes, const int *nlev_nod, int nEdges, const int *nlev_elem, int nl,
                      const int *edges, const int *edge_tri, double *LO, const double *adf_v,
                      const double *adf_h, double dt, const double *area, const double *hnode_new);

static void *xmalloc(size_t n)
{
    void *p = malloc(n ? n : 1);
    if (!p) {
        fprintf(stderr, "out of memory\n");
        exit(2);
    }
    return p;
}
#define ALLOC(T, n) ((T *)xmalloc(sizeof(T) * (size_t)(n)))

static int run(int nx, int ny, int nl, int full_depth)
{
    int64_t N, T, E;
    int dim;
    synth_mesh_sizes(nx, ny, &N, &T, &E, &dim);
    const int L = nl - 1;
    int *en = ALLOC(int, 3 * T), *ed = ALLOC(int, 2 * E), *et = ALLOC(int, 2 * E);
    int *nien = ALLOC(int, N), *nie = ALLOC(int, dim * N), *nle = ALLOC(int, T), *nln = ALLOC(int, N);
    if (synth_mesh_build(nx, ny, nl, 42, full_depth, en, ed, et, nien, nie, nle, nln)) return 1;
    double *ttf = ALLOC(double, N * L), *LO = ALLOC(double, N * L), *tmax = ALLOC(double, N * L);
    double *tmin = ALLOC(double, N * L), *plus = ALLOC(double, N * L), *minus = ALLOC(double, N * L);
    double *hn = ALLOC(double, N * L), *hnn = ALLOC(double, N * L), *dv = ALLOC(double, N * L);
    double *dh = ALLOC(double, N * L), *adfv = ALLOC(double, N * nl), *area = ALLOC(double, N * nl);
    double *ainv = ALLOC(double, N * nl), *adfh = ALLOC(double, E * L), *uv = ALLOC(double, 2 * L * T);
    double *adfv2 = ALLOC(double, N * nl), *adfh2 = ALLOC(double, E * L);
    synth_fill(43, 1, 1, N, L, NULL, 0.0, 1.0, ttf);
    synth_fill(43, 2, 1, N, L, NULL, 0.0, 1.0, LO);
    synth_fill(43, 3, 1, N, nl, NULL, 0.0, 0.5, adfv);
    synth_fill(43, 4, 1, E, L, NULL, 0.0, 0.5, adfh);
    synth_fill(43, 5, 0, N, nl, NULL, 0.5, 2.0, area);
    synth_fill(43, 6, 0, N, L, NULL, 5.0, 50.0, hn);
    synth_fill(43, 7, 0, N, L, NULL, 5.0, 50.0, hnn);
    synth_fill(43, 8, 1, N, L, NULL, 0.0, 1.0, dv);
    synth_fill(43, 9, 1, N, L, NULL, 0.0, 1.0, dh);
    for (int64_t i = 0; i < N * nl; i++) ainv[i] = 1.0 / area[i];
    for (int64_t i = 0; i < N * nl; i++) adfv2[i] = 0.0;
    for (int64_t i = 0; i < E * L; i++) adfh2[i] = 0.0;
    int st = oracle_full_pass(tmax, tmin, plus, minus, ttf, LO, adfv, adfh, uv, area, ainv, hn, hnn, dv, dh,
                              (int)N, 0, (int)T, (int)E, nl, nln, nle, en, nien, nie, dim, ed, et, 1, 1e-16,
                              1e3, 1.0);
    /* iter_yn branch on the limited fluxes (exercises the adf2 and LO-update indexing) */
    oracle_b3v((int)N, nln, nl, adfv, plus, minus, adfv2);
    oracle_b3h((int)E, nle, nl, ed, et, adfh, plus, minus, adfh2);
    oracle_lo_update((int)N, nln, (int)E, nle, nl, ed, et, LO, adfv, adfh, 1.0, area, hnn);
    int bad = 0;
    for (int64_t n = 0; n < N; n++)
        for (int z = 0; z < nln[n] - 1; z++)
            bad += !isfinite(dv[n * L + z]) || !isfinite(dh[n * L + z]) || !isfinite(LO[n * L + z]);
    printf("%dx%dx%d full_depth=%d: alg_state %d, non-finite %d\n", nx, ny, nl, full_depth, st, bad);
    free(en); free(ed); free(et); free(nien); free(nie); free(nle); free(nln);
    free(ttf); free(LO); free(tmax); free(tmin); free(plus); free(minus); free(hn); free(hnn); free(dv);
    free(dh); free(adfv); free(area); free(ainv); free(adfh); free(uv); free(adfv2); free(adfh2);
    return (st == 9 || st == 5) && bad == 0 ? 0 : 1;
}

int main(void)
{
    int rc = 0;
    rc |= run(16, 8, 11, 0);
    rc |= run(24, 12, 15, 1);
    rc |= run(5, 3, 3, 0);   /* minimum levels */
    rc |= run(33, 7, 48, 0); /* odd level count */
    return rc;
}
