/*
 * oracle/gustavson.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * CPU restatement of the algorithm the reference uses as its CPU comparator and test truth
 * for CSR x CSR SpGEMM:
 *   - reference call site: SpGEMM_vs_SpMV/profiler.py:408 (`A_fmt @ B_fmt`, scipy CSR@CSR) and
 *     the upstream truth `alpha * self.a.dot(self.b)` in
 *     modify_src/cupy-src/tests/cupyx_tests/test_cusparse.py:405-411;
 *   - third-party algorithm restated here: scipy 1.15.3 `sparsetools/csr.h`
 *     `csr_matmat_maxnnz` + `csr_matmat` (Gustavson / SMMP, reached from
 *     scipy/sparse/_compressed.py:546-590).  scipy is not part of /root/reference; its
 *     published algorithm is restated, and the restatement is pinned bit-exactly against
 *     scipy outputs committed as golden vectors under tests/golden/ (see
 *     tests/golden/make_golden.py and tests/test_oracle.py).
 *
 * Semantics restated exactly:
 *   * per output row i, A's entries are visited in stored order (jj ascending), and for
 *     each, B row Aj[jj]'s entries in stored order (kk ascending);
 *   * the accumulator starts at 0 and every product is formed and rounded on its own
 *     (`sums[k] += v*Bx[kk]`: one multiply, one add, NO fused multiply-add -- this file
 *     must be compiled with -ffp-contract=off);
 *   * scipy drops entries whose final sum is exactly 0 (keep_zeros=0); cuSPARSE / CuPy keep
 *     every structural entry (keep_zeros=1) -- both are available because the reference's
 *     GPU boundary (cusparseSpGEMM, cupyx/cusparse.py:2007-2142) keeps structural entries
 *     while its CPU comparator (scipy) drops them;
 *   * scipy emits a row's columns in linked-list order (last first-touched column first);
 *     sort=1 sorts each row by column (values move with their columns, unchanged).
 *
 * alpha is applied after accumulation (C = alpha * (A.B)), matching how the upstream test
 * forms its expectation (`alpha * a.dot(b)`).
 *
 * No part of the shipped library links or calls this file.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

/* Value types.  Complex values follow scipy's sparsetools `complex_wrapper` (and numpy's
 * complex multiply for alpha * C): (a+bi)(c+di) = (ac - bd) + (ad + bc)i with every
 * product and every sum rounded on its own; a sum is "zero" when both parts are 0. */
typedef struct { float re, im; } orc_c64;
typedef struct { double re, im; } orc_c128;

#define REAL_OPS(T, SUF)                                                                    \
    static inline T mul_##SUF(T a, T b) { return a * b; }                                   \
    static inline T add_##SUF(T a, T b) { return a + b; }                                   \
    static inline int nz_##SUF(T a) { return a != 0; }                                      \
    static inline int one_##SUF(T a) { return a == (T)1; }                                  \
    static inline T zero_##SUF(void) { return (T)0; }
#define CPLX_OPS(T, SUF)                                                                    \
    static inline T mul_##SUF(T a, T b) {                                                   \
        T r; r.re = a.re * b.re - a.im * b.im; r.im = a.re * b.im + a.im * b.re; return r; } \
    static inline T add_##SUF(T a, T b) { T r; r.re = a.re + b.re; r.im = a.im + b.im; return r; } \
    static inline int nz_##SUF(T a) { return a.re != 0 || a.im != 0; }                     \
    static inline int one_##SUF(T a) { return a.re == 1 && a.im == 0; }                     \
    static inline T zero_##SUF(void) { T r; r.re = 0; r.im = 0; return r; }
REAL_OPS(float, f32)
REAL_OPS(double, f64)
CPLX_OPS(orc_c64, c64)
CPLX_OPS(orc_c128, c128)

/* P = number of scalar products = sum over A entries of nnz(B row) (cusparseSpGEMM_getNumProducts). */
int64_t orc_num_products(int64_t n_row, const int64_t *Ap, const int32_t *Aj, const int64_t *Bp)
{
    int64_t p = 0;
    for (int64_t i = 0; i < n_row; ++i)
        for (int64_t jj = Ap[i]; jj < Ap[i + 1]; ++jj) p += Bp[Aj[jj] + 1] - Bp[Aj[jj]];
    return p;
}

/* Structural nnz per row (csr_matmat_maxnnz).  Writes Cp[0..n_row] (exclusive scan) and
 * returns nnz(C) with structural zeros kept.  Returns -1 on allocation failure. */
int64_t orc_symbolic(int64_t n_row, int64_t n_col, const int64_t *Ap, const int32_t *Aj,
                     const int64_t *Bp, const int32_t *Bj, int64_t *Cp)
{
    int64_t *mask = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n_col > 0 ? n_col : 1));
    if (!mask) return -1;
    for (int64_t c = 0; c < n_col; ++c) mask[c] = -1;
    int64_t nnz = 0;
    Cp[0] = 0;
    for (int64_t i = 0; i < n_row; ++i) {
        int64_t row_nnz = 0;
        for (int64_t jj = Ap[i]; jj < Ap[i + 1]; ++jj) {
            int32_t j = Aj[jj];
            for (int64_t kk = Bp[j]; kk < Bp[j + 1]; ++kk) {
                int32_t k = Bj[kk];
                if (mask[k] != i) { mask[k] = i; ++row_nnz; }
            }
        }
        nnz += row_nnz;
        Cp[i + 1] = nnz;
    }
    free(mask);
    return nnz;
}

/* Sort one row's (col, val) pairs by column; insertion sort for short rows, heap-free
 * merge via a scratch buffer otherwise.  Columns within a row are distinct. */
#define DEFINE_ROW_SORT(T, SUF)                                                             \
    static void row_sort_##SUF(int32_t *cj, T *cx, int64_t n, int32_t *tj, T *tx)          \
    {                                                                                       \
        if (n < 2) return;                                                                  \
        if (n <= 32) {                                                                      \
            for (int64_t a = 1; a < n; ++a) {                                               \
                int32_t kj = cj[a]; T kx = cx[a]; int64_t b = a - 1;                        \
                while (b >= 0 && cj[b] > kj) { cj[b + 1] = cj[b]; cx[b + 1] = cx[b]; --b; } \
                cj[b + 1] = kj; cx[b + 1] = kx;                                             \
            }                                                                               \
            return;                                                                         \
        }                                                                                   \
        int64_t h = n / 2;                                                                  \
        row_sort_##SUF(cj, cx, h, tj, tx);                                                  \
        row_sort_##SUF(cj + h, cx + h, n - h, tj, tx);                                      \
        int64_t a = 0, b = h, o = 0;                                                        \
        while (a < h && b < n) {                                                            \
            if (cj[a] <= cj[b]) { tj[o] = cj[a]; tx[o++] = cx[a++]; }                       \
            else { tj[o] = cj[b]; tx[o++] = cx[b++]; }                                      \
        }                                                                                   \
        while (a < h) { tj[o] = cj[a]; tx[o++] = cx[a++]; }                                 \
        while (b < n) { tj[o] = cj[b]; tx[o++] = cx[b++]; }                                 \
        memcpy(cj, tj, sizeof(int32_t) * (size_t)n);                                        \
        memcpy(cx, tx, sizeof(T) * (size_t)n);                                              \
    }

/* One output row, scipy csr_matmat body.  next/sums are n_col scratch arrays kept at
 * (-1, 0) between rows.  Returns the number of entries written. */
#define DEFINE_ROW(T, SUF)                                                                  \
    static int64_t row_matmat_##SUF(int64_t i, const int64_t *Ap, const int32_t *Aj,       \
                                    const T *Ax, const int64_t *Bp, const int32_t *Bj,      \
                                    const T *Bx, T alpha, int keep_zeros, int64_t *next,    \
                                    T *sums, int32_t *Cj, T *Cx)                            \
    {                                                                                       \
        int64_t head = -2, length = 0, w = 0;                                               \
        for (int64_t jj = Ap[i]; jj < Ap[i + 1]; ++jj) {                                    \
            int32_t j = Aj[jj];                                                             \
            T v = Ax[jj];                                                                   \
            for (int64_t kk = Bp[j]; kk < Bp[j + 1]; ++kk) {                                \
                int32_t k = Bj[kk];                                                         \
                T prod = mul_##SUF(v, Bx[kk]);                                              \
                sums[k] = add_##SUF(sums[k], prod);                                         \
                if (next[k] == -1) { next[k] = head; head = k; ++length; }                  \
            }                                                                               \
        }                                                                                   \
        for (int64_t q = 0; q < length; ++q) {                                              \
            if (keep_zeros || nz_##SUF(sums[head])) {                                       \
                Cj[w] = (int32_t)head;                                                      \
                Cx[w] = one_##SUF(alpha) ? sums[head] : mul_##SUF(alpha, sums[head]);       \
                ++w;                                                                        \
            }                                                                               \
            int64_t tmp = head;                                                             \
            head = next[head];                                                              \
            next[tmp] = -1;                                                                 \
            sums[tmp] = zero_##SUF();                                                       \
        }                                                                                   \
        return w;                                                                           \
    }

/* Full product.  Capacity of Cj/Cx must be >= orc_symbolic()'s result.  Writes Cp and
 * returns nnz(C) (after optional zero dropping), or -1 on allocation failure. */
#define DEFINE_SPGEMM(T, SUF)                                                               \
    DEFINE_ROW_SORT(T, SUF)                                                                 \
    DEFINE_ROW(T, SUF)                                                                      \
    int64_t orc_spgemm_##SUF(int64_t n_row, int64_t n_col, const int64_t *Ap,               \
                             const int32_t *Aj, const T *Ax, const int64_t *Bp,             \
                             const int32_t *Bj, const T *Bx, T alpha, int keep_zeros,       \
                             int sort, int64_t *Cp, int32_t *Cj, T *Cx)                     \
    {                                                                                       \
        size_t nc = (size_t)(n_col > 0 ? n_col : 1);                                        \
        int64_t *next = (int64_t *)malloc(sizeof(int64_t) * nc);                            \
        T *sums = (T *)calloc(nc, sizeof(T));                                               \
        int32_t *tj = (int32_t *)malloc(sizeof(int32_t) * nc);                              \
        T *tx = (T *)malloc(sizeof(T) * nc);                                                \
        if (!next || !sums || !tj || !tx) {                                                 \
            free(next); free(sums); free(tj); free(tx);                                     \
            return -1;                                                                      \
        }                                                                                   \
        for (size_t c = 0; c < nc; ++c) next[c] = -1;                                       \
        int64_t nnz = 0;                                                                    \
        Cp[0] = 0;                                                                          \
        for (int64_t i = 0; i < n_row; ++i) {                                               \
            int64_t w = row_matmat_##SUF(i, Ap, Aj, Ax, Bp, Bj, Bx, alpha, keep_zeros,      \
                                         next, sums, Cj + nnz, Cx + nnz);                   \
            if (sort) row_sort_##SUF(Cj + nnz, Cx + nnz, w, tj, tx);                        \
            nnz += w;                                                                       \
            Cp[i + 1] = nnz;                                                                \
        }                                                                                   \
        free(next); free(sums); free(tj); free(tx);                                         \
        return nnz;                                                                         \
    }                                                                                       \
    /* Multi-threaded variant (rows split over OpenMP threads; per-thread scratch).         \
     * Same arithmetic per row, so the output is identical to the serial one.  Used only    \
     * as the "fair multi-core CPU" point beside the single-threaded scipy comparator.      \
     * Cp must already hold the structural row pointer from orc_symbolic; rows are written  \
     * at those offsets (keep_zeros=1 layout) -- zero dropping is not offered here. */      \
    int64_t orc_spgemm_omp_##SUF(int64_t n_row, int64_t n_col, const int64_t *Ap,           \
                                 const int32_t *Aj, const T *Ax, const int64_t *Bp,         \
                                 const int32_t *Bj, const T *Bx, T alpha, int sort,         \
                                 int nthreads, const int64_t *Cp, int32_t *Cj, T *Cx)       \
    {                                                                                       \
        int failed = 0;                                                                     \
        size_t nc = (size_t)(n_col > 0 ? n_col : 1);                                        \
        (void)nthreads;                                                                     \
        _Pragma("omp parallel num_threads(nthreads) reduction(|:failed)")                   \
        {                                                                                   \
            int64_t *next = (int64_t *)malloc(sizeof(int64_t) * nc);                        \
            T *sums = (T *)calloc(nc, sizeof(T));                                           \
            int32_t *tj = (int32_t *)malloc(sizeof(int32_t) * nc);                          \
            T *tx = (T *)malloc(sizeof(T) * nc);                                            \
            if (!next || !sums || !tj || !tx) failed = 1;                                   \
            else {                                                                          \
                for (size_t c = 0; c < nc; ++c) next[c] = -1;                               \
                _Pragma("omp for schedule(dynamic, 64)")                                    \
                for (int64_t i = 0; i < n_row; ++i) {                                       \
                    int64_t w = row_matmat_##SUF(i, Ap, Aj, Ax, Bp, Bj, Bx, alpha, 1, next, \
                                                 sums, Cj + Cp[i], Cx + Cp[i]);             \
                    if (sort) row_sort_##SUF(Cj + Cp[i], Cx + Cp[i], w, tj, tx);            \
                }                                                                           \
            }                                                                               \
            free(next); free(sums); free(tj); free(tx);                                     \
        }                                                                                   \
        return failed ? -1 : Cp[n_row];                                                     \
    }

DEFINE_SPGEMM(double, f64)
DEFINE_SPGEMM(float, f32)
DEFINE_SPGEMM(orc_c64, c64)
DEFINE_SPGEMM(orc_c128, c128)

/* Canonical-format check (restates cupyx _has_canonical_format_kern,
 * modify_src/cupy-src/cupyx/scipy/sparse/_compressed.py:177-192): indptr non-decreasing
 * and, within each row, indices strictly increasing. */
int orc_has_canonical_format(int64_t n_row, const int64_t *Ap, const int32_t *Aj)
{
    for (int64_t i = 0; i < n_row; ++i) {
        if (Ap[i + 1] < Ap[i]) return 0;
        for (int64_t jj = Ap[i] + 1; jj < Ap[i + 1]; ++jj)
            if (Aj[jj - 1] >= Aj[jj]) return 0;
    }
    return 1;
}

/* CSR x dense vector (scipy `csr_matvec`, reached from csr_matrix @ ndarray -> _mul_vector,
 * the SpMV half of SpGEMM_vs_SpMV/profiler.py:410-411): y[i] = ((0 + a_i0 x_j0) + a_i1 x_j1)
 * + ..., every product and sum rounded on its own, A's entries in stored order; then
 * y = alpha * y when alpha != 1 (numpy's scalar multiply). */
#define DEFINE_SPMV(T, SUF)                                                                 \
    void orc_spmv_##SUF(int64_t n_row, const int64_t *Ap, const int32_t *Aj, const T *Ax,   \
                        const T *x, T alpha, T *y)                                          \
    {                                                                                       \
        for (int64_t i = 0; i < n_row; ++i) {                                               \
            T sum = zero_##SUF();                                                           \
            for (int64_t jj = Ap[i]; jj < Ap[i + 1]; ++jj)                                  \
                sum = add_##SUF(sum, mul_##SUF(Ax[jj], x[Aj[jj]]));                         \
            y[i] = one_##SUF(alpha) ? sum : mul_##SUF(alpha, sum);                          \
        }                                                                                   \
    }
DEFINE_SPMV(double, f64)
DEFINE_SPMV(float, f32)
DEFINE_SPMV(orc_c64, c64)
DEFINE_SPMV(orc_c128, c128)
