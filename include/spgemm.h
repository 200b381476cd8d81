/*
 * spgemm.h -- C ABI of libmi355_spgemm.so, the MI355X (gfx950) CSR x CSR SpGEMM engine.
 *
 * Drop-in boundary for the reference's hot path.  Each entry point names the reference
 * interface it replaces (paths relative to the reference repository root;
 * "cupy-src/" = modify_src/cupy-src/).  The reference reaches closed NVIDIA cuSPARSE through
 * two callers, and both map onto this header:
 *
 *   * native drivers  cupy_cusparse/spgemm_from_txt_alg{1,2,3}.cu:145-206
 *       cusparseCreate / cusparseCreateCsr / cusparseSpGEMM_workEstimation /
 *       cusparseSpGEMM_estimateMemory / cusparseSpGEMM_compute / cusparseSpMatGetSize /
 *       cusparseCsrSetPointers / cusparseSpGEMM_copy / cusparseDestroy
 *   * CuPy wrapper    cupy-src/cupyx/cusparse.py:2007-2142 `spgemm(a, b, alpha, alg,
 *       chunk_fraction)` through the Cython bindings cupy-src/cupy_backends/cuda/libs/
 *       cusparse.pyx:5063-5152 (spGEMM_createDescr/workEstimation/compute/copy/
 *       estimateMemory[_getBuf3]).
 *
 * Conventions:
 *   - Plain C types only: device pointers as void*, sizes as int64_t/size_t.  No HIP or C++
 *     types appear in the signatures (a hipStream_t is passed as void*).
 *   - Ownership: the caller owns A, B, C and the workspace (the cuSPARSE convention).  The
 *     library never frees caller memory; a plan owns only small host metadata plus the
 *     caller-provided workspace pointer.
 *   - Two-call size query: spg_plan(..., ws = NULL) returns the workspace size, then
 *     spg_plan(..., ws = buffer) builds the plan (like workEstimation / compute with a NULL
 *     buffer).  C's row pointer is written by spg_symbolic, which returns nnz(C) to the
 *     host; the caller then allocates C's indices/values and calls spg_numeric (like
 *     cusparseSpMatGetSize -> cusparseCsrSetPointers -> cusparseSpGEMM_copy).
 *   - Stream ordering: every call enqueues on the handle's stream.  The only calls that
 *     wait on the device are spg_plan for ALG3 (its chunk plan reads the product-count
 *     prefix back) and for ALG1 on shapes outside the short-row kernel (the upper-bound
 *     buffer is sized from the product count), spg_num_products, spg_symbolic (nnz(C) to
 *     host) and spg_validate_csr.  spg_plan for ALG1 on short-row shapes does no device work
 *     (its output buffer is sized from the expected product count).  spg_symbolic waits
 *     only for nnz(C): under ALG1 it returns while the numeric pass it queued is still
 *     running, so C is ready in stream order, not on return.
 *   - Errors are status codes only; the library never calls exit().  SPG_STATUS_ALLOC_FAILED
 *     lets a harness print "[SKIP]" (dense_vs_sparseGEMM/utils.py:156-173).
 *   - A handle is not thread-safe: one handle per host thread per device (mirrors CuPy's
 *     thread-local handles, cupy-src/cupy/cuda/device.pyx:228-243).
 *   - Numerics: C = alpha * (A.B).  Each C(i,j) is accumulated in A's stored entry order,
 *     every product and sum separately rounded (no FMA), starting from 0, then scaled by
 *     alpha once when alpha != 1.  That is exactly scipy's csr_matmat rule, so results are
 *     bit-identical to scipy after dropping exact zeros and sorting columns, and identical
 *     from run to run.  Structural entries are kept (cuSPARSE semantics): an entry whose
 *     sum cancels to 0 is stored as an explicit 0.  C's columns are sorted ascending.
 */
#ifndef MI355_SPGEMM_H
#define MI355_SPGEMM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPG_VERSION_MAJOR 0
#define SPG_VERSION_MINOR 2
#define SPG_VERSION_PATCH 0

/* Status codes.  0..11 keep the numeric values of cusparseStatus_t so the drivers' error
 * lines read the same (CHECK_CUSPARSE in cupy_cusparse/spgemm_from_txt_alg1.cu:15-17). */
typedef enum {
    SPG_STATUS_SUCCESS = 0,
    SPG_STATUS_NOT_INITIALIZED = 1,
    SPG_STATUS_ALLOC_FAILED = 2,
    SPG_STATUS_INVALID_VALUE = 3,
    SPG_STATUS_ARCH_MISMATCH = 4,
    SPG_STATUS_EXECUTION_FAILED = 6,
    SPG_STATUS_INTERNAL_ERROR = 7,
    SPG_STATUS_NOT_SUPPORTED = 10,
    SPG_STATUS_INSUFFICIENT_RESOURCES = 11,
    SPG_STATUS_OVERFLOW = 100,  /* nnz(C) does not fit C's row-pointer type            */
    SPG_STATUS_HIP_ERROR = 101  /* a HIP runtime call failed; see spg_last_hip_error   */
} spg_status_t;

/* Index type of a row pointer (indptr).  Column indices are always int32. */
typedef enum { SPG_INDEX_32I = 32, SPG_INDEX_64I = 64 } spg_index_t;

/* Value type.  Numbers equal cudaDataType's CUDA_R_32F / CUDA_R_64F / CUDA_C_32F /
 * CUDA_C_64F (cupyx/cusparse.py takes f32/f64/c64/c128, test_cusparse.py:372-375).
 * Complex values are (real, imag) pairs, numpy's layout; alpha then points to one pair. */
typedef enum { SPG_R_32F = 0, SPG_R_64F = 1, SPG_C_32F = 4, SPG_C_64F = 5 } spg_dtype_t;

/* Algorithm selector (cusparseSpGEMMAlg_t roles, cupy-src/cupy_backends/cuda/libs/
 * cusparse.pxd:158-164; chosen at cupy-src/cupyx/cusparse.py:2052-2057):
 *   SPG_ALG_DEFAULT  library choice (currently ALG2);
 *   SPG_ALG1  one numeric pass, one host sync: on short-row shapes a count pass (nnz per
 *             row) and ONE numeric launch that also scans the counts into C's row pointer
 *             and writes C compact into an estimate-sized workspace buffer (an output past
 *             the estimate is redone two-phase into C); spg_numeric then copies/scales it
 *             (or only scales, when C's arrays are that buffer: spg_result_in_workspace).
 *             Other shapes: a single pass into an upper-bound buffer (workspace ~
 *             num_products) that spg_numeric compacts, or (tile path) two phases -- the
 *             memory-hungry / fewest-passes point, like cuSPARSE ALG1;
 *   SPG_ALG2  two phase: symbolic (nnz per row) then numeric straight into C; workspace is
 *             O(rows + nnz(A));
 *   SPG_ALG3  two phase, numeric run in row chunks so each chunk touches at most
 *             chunk_fraction of the products and the per-chunk workspace is capped (the
 *             ALG3 role: bounded working set at some extra launch cost). */
typedef enum { SPG_ALG_DEFAULT = 0, SPG_ALG1 = 1, SPG_ALG2 = 2, SPG_ALG3 = 3 } spg_alg_t;

/* CSR view of caller-owned device memory (cusparseCreateCsr, spgemm_from_txt_alg1.cu:
 * 150-160; SpMatDescriptor.create, cupy-src/cupyx/cusparse.py:1295-1325).  Zero-based.
 * indptr has rows+1 entries of indptr_type; indices has nnz int32 entries; values has nnz
 * entries of value_type.  nnz must equal indptr[rows] (not checked on the device). */
typedef struct {
    int64_t rows;
    int64_t cols;
    int64_t nnz;
    void *indptr;
    void *indices;
    void *values;
    spg_index_t indptr_type;
    spg_dtype_t value_type;
} spg_csr_t;

typedef struct spg_handle_s *spg_handle_t;
typedef struct spg_plan_s *spg_plan_t;

/* Library version as MAJOR*10000 + MINOR*100 + PATCH (cusparseGetVersion). */
int spg_version(void);

/* Build stamp of the loaded library: "source_id=<16 hex> hipflags=<flags>", the id being a
 * hash of the sources and the compile flags it was built from (spmm_amd/source_id.py).
 * Measurements are stamped with it.  No cuSPARSE counterpart. */
const char *spg_build_info(void);

/* Human-readable status name (cusparseGetErrorString). */
const char *spg_status_string(spg_status_t status);

/* Handle lifecycle (cusparseCreate / cusparseDestroy, spgemm_from_txt_alg1.cu:145,205).
 * The handle binds to `hip_device`; -1 keeps the calling thread's current device. */
spg_status_t spg_create(spg_handle_t *handle, int hip_device);
spg_status_t spg_destroy(spg_handle_t handle);

/* Stream for all subsequent work (cusparseSetStream).  `stream` is a hipStream_t; NULL is
 * the null stream.  A change of stream first drains the old one. */
spg_status_t spg_set_stream(spg_handle_t handle, void *stream);

/* Last HIP error code seen by this handle (0 if none), for SPG_STATUS_HIP_ERROR. */
int spg_last_hip_error(spg_handle_t handle);

/* Plan C = A.B (cusparseSpGEMM_workEstimation x2 + cusparseSpGEMM_estimateMemory x2,
 * cupy-src/cupyx/cusparse.py:2061-2105; spgemm_from_txt_alg3.cu:170-202).
 *   A: m x k, B: k x n, both canonical CSR (sorted, duplicate-free rows, the reference's
 *   `assert a.has_canonical_format`, cupy-src/cupyx/cusparse.py:2030-2031), same value
 *   type, same indptr type.
 *   chunk_fraction in (0, 1] is used by ALG3 (ignored otherwise, as cuSPARSE ignores it
 *   for ALG2); out of range -> SPG_STATUS_INVALID_VALUE.
 *   workspace == NULL: size query, *workspace_bytes is set, *plan is left untouched.
 *   workspace != NULL: *workspace_bytes must be >= the queried size; *plan is created.
 * The plan keeps the A and B descriptors by value: their device arrays must stay alive
 * and unchanged until spg_numeric has completed. */
spg_status_t spg_plan(spg_handle_t handle, const spg_csr_t *A, const spg_csr_t *B,
                      spg_alg_t alg, float chunk_fraction, size_t *workspace_bytes,
                      void *workspace, spg_plan_t *plan);

/* Number of scalar products P = sum over A's entries of nnz(B row)
 * (cusparseSpGEMM_getNumProducts, cupy-src/cupy_backends/cuda/libs/cusparse.pxd:73;
 * spgemm_from_txt_alg3.cu:190-192).  GFLOPS = 2P / t.  Waits for the device. */
spg_status_t spg_num_products(spg_handle_t handle, spg_plan_t plan, int64_t *num_products);

/* Symbolic phase: writes C's row pointer (rows(A)+1 entries of C_indptr_type) and returns
 * nnz(C) on the host (cusparseSpGEMM_compute + cusparseSpMatGetSize,
 * cupy-src/cupyx/cusparse.py:2108-2127; spgemm_from_txt_alg1.cu:177-183).  nnz(C) counts
 * structural entries.  SPG_STATUS_OVERFLOW if it does not fit C_indptr_type. */
spg_status_t spg_symbolic(spg_handle_t handle, spg_plan_t plan, void *C_indptr,
                          spg_index_t C_indptr_type, int64_t *nnzC);

/* Numeric phase: fills C->indices and C->values (caller-allocated, nnzC entries) with
 * alpha*A.B; C->indptr must be the array spg_symbolic wrote.  `alpha` points to one host
 * value of C's value type (CUSPARSE_POINTER_MODE_HOST, spgemm_from_txt_alg1.cu:146;
 * beta is always 0).  (cusparseCsrSetPointers + cusparseSpGEMM_copy,
 * cupy-src/cupyx/cusparse.py:2128-2137.)  Stream-ordered; does not wait. */
spg_status_t spg_numeric(spg_handle_t handle, spg_plan_t plan, const void *alpha,
                         spg_csr_t *C);

/* Sparse matrix x dense vector: y = alpha * A x + beta * y (A CSR, x of A.cols entries,
 * y of A.rows entries, all of A's value type; alpha/beta host values).  Each row is summed
 * in A's entry order from 0, so the result equals scipy's csr_matvec bit for bit (beta = 0,
 * alpha = 1).  Stream-ordered; does not wait.  (cusparseSpMV as called by
 * cupyx.cusparse.spmv, modify_src/cupy-src/cupyx/cusparse.py:1373-1432; the SpMV half of
 * SpGEMM_vs_SpMV/profiler.py:410-411.) */
spg_status_t spg_spmv(spg_handle_t handle, const spg_csr_t *A, const void *x, const void *alpha,
                      const void *beta, void *y);

/* ALG1 single pass: after spg_symbolic, C's column indices and values may already sit
 * compact in the workspace (nnzC entries at *indices / *values; NULL otherwise).  A
 * caller may hand exactly these pointers to spg_numeric as C->indices / C->values: the
 * numeric call then only scales by alpha in place (once) instead of copying.  No
 * cuSPARSE counterpart; ignoring it keeps the cuSPARSE call sequence (a copy). */
spg_status_t spg_result_in_workspace(spg_plan_t plan, void **indices, void **values);

/* Bytes this multiply needs on the device beyond its inputs: workspace + C's three arrays
 * (the "peak HBM bytes" metric; inputs excluded like the reference's inputs-on-GPU
 * ΔPeak, dense_vs_sparseGEMM/utils.py:243-250).  Exact once spg_symbolic has run; before
 * that C is counted with nnz(C) <= num_products as an upper bound. */
spg_status_t spg_peak_bytes(spg_plan_t plan, size_t *bytes);

/* Device check that M is canonical CSR: indptr non-decreasing and indices strictly
 * increasing inside every row, and every index in [0, cols) (replaces CuPy's
 * _has_canonical_format_kern, cupy-src/cupyx/scipy/sparse/_compressed.py:177-192, plus the
 * bounds check of validate_csr_indices, spgemm_from_txt_alg1.cu:80-102).
 * *is_canonical = 1 canonical, 0 sorted-order or duplicate violation, -1 index out of
 * bounds or bad indptr.  Waits for the device. */
spg_status_t spg_validate_csr(spg_handle_t handle, const spg_csr_t *M, int *is_canonical);

/* What a plan will run (a diagnostic for tests and profilers; no cuSPARSE counterpart, the
 * closest being the chunk plan cusparseSpGEMM_estimateMemory makes internally,
 * spgemm_from_txt_alg3.cu:195-202).  path: 0 general windowed kernels, 1 short-row kernel,
 * 2 tile path (tile_width columns per numeric tile, tiles_per_row tiles, dense_tiles 1
 * when the accumulator is addressed by column).  n_chunks row chunks (ALG3: the chunk
 * cut; otherwise 1); their n_chunks + 1 row boundaries go to chunk_rows (at most
 * `capacity` entries written; chunk_rows may be NULL when capacity is 0).  lds_ordered 1
 * when fp64 / complex128 tiles run the ordered-LDS-add kernels -- the handle's device check at
 * spg_create found the ordering they rely on -- and 0 when they fall back to owner rounds
 * (same results).  record_group (tile path): numeric tiles per VALUE TILE -- B's records are
 * laid out per group of that many adjacent tiles (1: plain tile-major); the value-tile API
 * below works in value tiles of tile_width * record_group columns, ceil(tiles_per_row /
 * record_group) of them. */
typedef struct {
    int path;
    int tile_width;
    int64_t tiles_per_row;
    int dense_tiles;
    int64_t n_chunks;
    int lds_ordered;
    int record_group;
} spg_plan_info_t;
spg_status_t spg_plan_info(spg_plan_t plan, spg_plan_info_t *info, int64_t *chunk_rows, int64_t capacity);

/* Free a plan's host metadata (cusparseSpGEMM_destroyDescr).  Never touches the
 * caller's workspace. */
spg_status_t spg_plan_destroy(spg_plan_t plan);

/* The whole call sequence of cupyx.cusparse.spgemm (cupy-src/cupyx/cusparse.py:2041-2142:
 * workEstimation/estimateMemory -> compute -> getSize -> copy) in ONE call, for a caller
 * that holds the workspace spg_plan's size query asked for (same A, B, alg,
 * chunk_fraction).  Writes C's row pointer (rows(A)+1 entries of C_indptr_type;
 * SPG_STATUS_OVERFLOW when int32 cannot hold nnz(C): call again with an int64 array) and
 * nnz(C) to *nnzC (the call's one host sync).
 *   When C's columns and values sit compact in the workspace (ALG1), they are scaled by
 *   *alpha in place, *C_indices / *C_values point at them (nnzC entries) and *plan_out is
 *   NULL: the product is complete (stream-ordered).
 *   Otherwise *C_indices / *C_values are NULL and *plan_out is the live plan: the caller
 *   allocates C's arrays (nnzC entries) and finishes with spg_numeric + spg_plan_destroy.
 * *peak_bytes is the spg_peak_bytes figure for this product.  No cuSPARSE counterpart: it
 * removes four host round trips per product from a binding's call path. */
spg_status_t spg_spgemm_ws(spg_handle_t handle, const spg_csr_t *A, const spg_csr_t *B, spg_alg_t alg,
                           float chunk_fraction, const void *alpha, void *workspace, size_t workspace_bytes,
                           void *C_indptr, spg_index_t C_indptr_type, int64_t *nnzC, void **C_indices,
                           void **C_values, size_t *peak_bytes, spg_plan_t *plan_out);

/* Numeric phase by column-tile groups, for a B whose VALUES arrive in pieces (the multi-GPU
 * row-block step: B's structure is broadcast first, its values follow group by group and
 * each group's numeric tiles start as soon as its values land -- the reference broadcasts
 * a sparse matrix as three grouped payloads, modify_src/cupy-src/cupyx/distributed/
 * _nccl_comm.py:651-674; no cuSPARSE counterpart: cusparseSpGEMM_compute needs all of B).
 * Tile-path plans with one row chunk only (spg_plan_info: path 2, n_chunks 1); anything
 * else returns SPG_STATUS_NOT_SUPPORTED and the caller takes spg_numeric.
 * The unit is the VALUE TILE: record_group adjacent numeric tiles (spg_plan_info), i.e. a
 * column range of tile_width * record_group columns; value_tiles = ceil(tiles_per_row /
 * record_group).
 *   spg_tile_value_offsets: the value_tiles + 1 offsets (entries) of each value tile's
 *     values in TILE-MAJOR order -- B's entries with columns in value tile 0 row by row,
 *     then value tile 1, ...  One device->host copy.  The order depends only on B's
 *     structure and the value-tile width, so plans on different devices with equal widths
 *     agree.  Valid right after spg_plan: the first of these calls (or spg_symbolic) builds
 *     the plan's tile layout from B's structure, so the values can be sent while the
 *     symbolic pass runs.
 *   spg_tile_values: B's values (row-major, B->values of the plan) permuted into that
 *     order (nnz(B) entries of B's value type) -- on the device that holds them.
 *   spg_numeric_tiles: C's entries in columns of value tiles [tile_begin, tile_end) from the
 *     tile-major values (only that range of them is read), after spg_symbolic, stream-
 *     ordered like spg_numeric.  Calls over disjoint ranges covering every value tile give
 *     C bit for bit as spg_numeric does; the plan's B->values is never read. */
spg_status_t spg_tile_value_offsets(spg_handle_t handle, spg_plan_t plan, int64_t *offsets, int64_t capacity);
spg_status_t spg_tile_values(spg_handle_t handle, spg_plan_t plan, void *tile_major_values);
spg_status_t spg_numeric_tiles(spg_handle_t handle, spg_plan_t plan, const void *alpha, spg_csr_t *C,
                               const void *tile_major_values, int64_t tile_begin, int64_t tile_end);

/* B's column indices in 16 bits, for the multi-GPU structure broadcast (spmm_amd.
 * distributed.broadcast_csr; no cuSPARSE counterpart -- the reference broadcasts B's int32
 * indices as they are, modify_src/cupy-src/cupyx/distributed/_nccl_comm.py:651-674).  The
 * columns of M are cut into blocks of 65536; per row, the ceil(cols / 65536) - 1 interior
 * block starts (the offset from the row's start of its first entry with column >= c * 65536,
 * or the row's length, for c = 1, 2, ...; uint32, row-major) plus the low 16 bits of every
 * column carry the indices exactly, in 2 bytes per entry + 4 per row and interior block
 * (config 5's B: 141 MB instead of 276 MB).  M canonical (rows sorted); stream-ordered.
 *   spg_cols16_split: M's indptr/indices -> block_starts, lo16 (nnz entries).  block_starts
 *     may be NULL for M at most 65536 columns wide.  M->values is not read.
 *   spg_cols16_join: block_starts, lo16 and M's indptr -> M->indices. */
spg_status_t spg_cols16_split(spg_handle_t handle, const spg_csr_t *M, uint32_t *block_starts, uint16_t *lo16);
spg_status_t spg_cols16_join(spg_handle_t handle, spg_csr_t *M, const uint32_t *block_starts, const uint16_t *lo16);

/* Per-phase device timing: with timing enabled every kernel the handle launches is
 * bracketed by hipEvents on the handle's stream, and spg_get_timing returns the
 * accumulated device milliseconds and launch counts per phase (the build's equivalent of
 * the reference's per-run wall clock, SpGEMM_alg_comparison/profiler.py:119-122, resolved
 * per kernel).  spg_set_timing resets the accumulators; spg_get_timing waits for the
 * device.  Off by default (events cost a few microseconds per launch). */
typedef enum {
    SPG_PHASE_PRODUCTS = 0,   /* k_row_products: P_i per row                      */
    SPG_PHASE_SCAN = 1,       /* k_scan_lb / k_items_to_rowptr: prefix sums       */
    SPG_PHASE_SYMBOLIC = 2,   /* k_row (count) / k_tile_sym(_seg) / k_symbolic     */
    SPG_PHASE_NUMERIC = 3,    /* k_row / k_tile_dn / k_tile_sp / k_tile /          */
                              /* k_numeric: values (ALG1 also structure); one       */
                              /* kernel per launch                                  */
    SPG_PHASE_COMPACT = 4,    /* k_compact: ALG1 copy into C                        */
    SPG_PHASE_VALIDATE = 5,   /* k_validate                                         */
    SPG_PHASE_SPILL = 6,      /* k_symbolic / k_numeric over the rows the short-row */
                              /* kernel handed on (list mode)                        */
    SPG_PHASE_SPMV = 7,       /* k_spmv                                             */
    SPG_PHASE_LAYOUT = 8,     /* the tile path's B re-layout: once per plan          */
                              /* (k_tile_index, k_bt_count, k_bj16, k_bt_pack) and   */
                              /* per tile group (k_bt_fill, spg_numeric_tiles)        */
    SPG_NUM_PHASES = 9
} spg_phase_t;

typedef struct {
    double ms[SPG_NUM_PHASES];
    int64_t launches[SPG_NUM_PHASES];
} spg_timing_t;

spg_status_t spg_set_timing(spg_handle_t handle, int enable);
spg_status_t spg_get_timing(spg_handle_t handle, spg_timing_t *timing);

#ifdef __cplusplus
}
#endif

#endif /* MI355_SPGEMM_H */
