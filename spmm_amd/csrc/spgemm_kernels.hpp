// spgemm_kernels.hpp -- gfx950 kernels of the SpGEMM engine (see spg_device.hpp for the
// row engine).  All kernels are templated on the value type T (float/double), the input
// row-pointer type IP (int32/int64, shared by A and B) and the output row-offset type.
#pragma once

#include "spg_device.hpp"

namespace spg {

constexpr int WPB = 4;              // waves per block
constexpr int BLOCK = WPB * WAVE;   // 256 threads

// ---------------------------------------------------------------------------------------
// P_i = number of products of output row i (workEstimation).  One wave per row.
template <typename IP>
__global__ __launch_bounds__(BLOCK) void k_row_products(int64_t rows, const IP* __restrict__ Ap,
                                                        const int32_t* __restrict__ Aj,
                                                        const IP* __restrict__ Bp,
                                                        int64_t* __restrict__ out) {
    const int l = lane_id();
    const int64_t row = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
    if (row >= rows) return;
    const int64_t a0 = Ap[row], a1 = Ap[row + 1];
    long long s = 0;
    for (int64_t jj = a0 + l; jj < a1; jj += WAVE) {
        const int32_t k = Aj[jj];
        s += (long long)(Bp[k + 1] - Bp[k]);
    }
    s = wave_sum64(s);
    if (l == 0) out[row] = s;
}

// ---------------------------------------------------------------------------------------
// Exclusive scan of in[0..n) into out[0..n], out[n] = total; scalars[0] = total,
// scalars[1] = 1 if the total does not fit OUT.  One block of 1024 threads, 8 items each.
template <typename OUT>
__global__ __launch_bounds__(1024) void k_scan_excl(int64_t n, const int64_t* __restrict__ in,
                                                    OUT* __restrict__ out,
                                                    int64_t* __restrict__ scalars) {
    constexpr int ITEMS = 8;
    __shared__ long long wsum[16];
    const int tid = threadIdx.x, l = lane_id(), w = tid >> 6;
    long long carry = 0;
    for (int64_t base = 0; base < n; base += 1024 * ITEMS) {
        long long v[ITEMS];
        long long tsum = 0;
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const int64_t idx = base + (int64_t)tid * ITEMS + j;
            v[j] = idx < n ? in[idx] : 0;
            tsum += v[j];
        }
        const long long incl = wave_incl_sum64(tsum);
        if (l == WAVE - 1) wsum[w] = incl;
        __syncthreads();
        long long wbase = 0, btot = 0;
        for (int q = 0; q < 16; ++q) {
            const long long x = wsum[q];
            if (q < w) wbase += x;
            btot += x;
        }
        long long run = carry + wbase + incl - tsum;
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const int64_t idx = base + (int64_t)tid * ITEMS + j;
            if (idx < n) out[idx] = (OUT)run;
            run += v[j];
        }
        carry += btot;
        __syncthreads();
    }
    if (tid == 0) {
        out[n] = (OUT)carry;
        scalars[0] = carry;
        scalars[1] = (sizeof(OUT) == 4 && carry > 2147483647LL) ? 1 : 0;
    }
}

// ---------------------------------------------------------------------------------------
// Symbolic phase: structural nnz of each output row (no values).  One wave per row, a
// private bitmap window in LDS.  Rows of C wider than one window walk B with cursors.
template <typename IP>
__global__ __launch_bounds__(BLOCK) void k_symbolic(
    int64_t row0, int64_t nrows, int64_t ncols, const IP* __restrict__ Ap,
    const int32_t* __restrict__ Aj, const IP* __restrict__ Bp, const int32_t* __restrict__ Bj,
    int64_t* __restrict__ row_cnt, uint32_t* __restrict__ cur, int64_t nz0) {
    __shared__ uint32_t lds[WPB][SymGeom::BYTES / 4];
    const int l = lane_id();
    const int wv = threadIdx.x >> 6;
    const int64_t row = row0 + (int64_t)blockIdx.x * WPB + wv;
    if (row >= row0 + nrows) return;
    uint32_t* bits = lds[wv];
    int* marker = (int*)(bits + SymGeom::NWMAX);
    const int64_t a0 = Ap[row], a1 = Ap[row + 1];
    long long total = 0;
    if (a0 < a1 && ncols > 0) {
        const bool single = ncols <= 32LL * SymGeom::NWMAX;
        for (int64_t lo = 0; lo < ncols;) {
            const int64_t hi = single ? ncols : min(ncols, lo + 32LL * SymGeom::NWMAX);
            const int nw = (int)((hi - lo + 31) >> 5);
            for (int w = l; w < nw; w += WAVE) bits[w] = 0u;
            wsync();
            for (int64_t b = a0; b < a1; b += WAVE) {
                const int64_t jj = b + l;
                if (single) {
                    long long beg = 0;
                    int cnt = 0;
                    if (jj < a1) {
                        const int32_t k = Aj[jj];
                        beg = Bp[k];
                        cnt = (int)(Bp[k + 1] - beg);
                    }
                    for_each_product(beg, cnt, marker, [&](bool v, int, long long idx) {
                        if (v) set_bit(bits, Bj[idx]);
                    });
                } else if (jj < a1) {
                    const int32_t k = Aj[jj];
                    const int64_t rb = Bp[k], re = Bp[k + 1];
                    int64_t p = rb + (lo == 0 ? 0 : (int64_t)cur[jj - nz0]);
                    while (p < re) {
                        int c[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) c[u] = (p + u < re) ? Bj[p + u] : 0x7fffffff;
                        int n = 0;
#pragma unroll
                        for (int u = 0; u < 4; ++u)
                            if (c[u] < hi) { set_bit(bits, (int)(c[u] - lo)); ++n; }
                        p += n;
                        if (n < 4) break;
                    }
                    cur[jj - nz0] = (uint32_t)(p - rb);
                }
            }
            wsync();
            long long cnt = 0;
            for (int w = l; w < nw; w += WAVE) cnt += __popc(bits[w]);
            total += wave_sum64(cnt);
            wsync();
            lo = hi;
        }
    }
    if (l == 0) row_cnt[row] = total;
}

// ---------------------------------------------------------------------------------------
// Numeric phase.  UB=false: rows are written at C's row pointer Coff (exact, from the
// symbolic phase).  UB=true (ALG1 single pass): rows are written at the product-count
// prefix Coff (an upper bound) and each row's nnz goes to row_cnt.
template <typename T, typename IP, typename OFF, bool UB>
__global__ __launch_bounds__(BLOCK) void k_numeric(
    int64_t row0, int64_t nrows, int64_t ncols, const IP* __restrict__ Ap,
    const int32_t* __restrict__ Aj, const T* __restrict__ Ax, const IP* __restrict__ Bp,
    const int32_t* __restrict__ Bj, const T* __restrict__ Bx, const OFF* __restrict__ Coff,
    int32_t* __restrict__ Cj, T* __restrict__ Cx, T alpha, int64_t* __restrict__ row_cnt,
    uint32_t* __restrict__ seg, int64_t nz0, int64_t seg_len) {
    using G = NumGeom<T>;
    __shared__ __attribute__((aligned(16))) char lds_raw[WPB][G::BYTES];
    const int l = lane_id();
    const int wv = threadIdx.x >> 6;
    const int64_t row = row0 + (int64_t)blockIdx.x * WPB + wv;
    if (row >= row0 + nrows) return;
    char* base = lds_raw[wv];
    T* acc = (T*)base;
    uint32_t* bits = (uint32_t*)(base + sizeof(T) * G::CAP);
    uint32_t* wpre = bits + G::NWMAX;
    uint32_t* tag = wpre + G::NWMAX;
    int* marker = (int*)(tag + G::CAP);
    uint32_t* seg_cur = seg;
    uint32_t* seg_end = seg + seg_len;

    const int64_t a0 = Ap[row], a1 = Ap[row + 1];
    const int64_t out0 = (int64_t)Coff[row];
    const int64_t est = (int64_t)Coff[row + 1] - out0;
    int64_t written = 0;
    if (a0 < a1 && ncols > 0 && est > 0) {
        const bool single = ncols <= 32LL * G::NWMAX && est <= G::CAP;
        int nw_def;
        if (single) {
            nw_def = (int)((ncols + 31) >> 5);
        } else {
            const double w = 0.75 * (double)G::CAP * (double)ncols / ((double)est * 32.0);
            nw_def = w < 1.0 ? 1 : (w > (double)G::NWMAX ? G::NWMAX : (int)w);
        }
        for (int64_t lo = 0; lo < ncols;) {
            int nw = (int)min((int64_t)nw_def, (ncols - lo + 31) >> 5);
            int64_t hi;
            int nnz_sw;
            for (;;) {
                hi = min(ncols, lo + 32LL * nw);
                for (int w = l; w < nw; w += WAVE) bits[w] = 0u;
                wsync();
                // ---- pass A: structure of the window
                for (int64_t b = a0; b < a1; b += WAVE) {
                    const int64_t jj = b + l;
                    if (single) {
                        long long beg = 0;
                        int cnt = 0;
                        if (jj < a1) {
                            const int32_t k = Aj[jj];
                            beg = Bp[k];
                            cnt = (int)(Bp[k + 1] - beg);
                        }
                        for_each_product(beg, cnt, marker, [&](bool v, int, long long idx) {
                            if (v) set_bit(bits, Bj[idx]);
                        });
                    } else if (jj < a1) {
                        const int32_t k = Aj[jj];
                        const int64_t rb = Bp[k], re = Bp[k + 1];
                        int64_t p = rb + (lo == 0 ? 0 : (int64_t)seg_cur[jj - nz0]);
                        while (p < re) {
                            int c[4];
#pragma unroll
                            for (int u = 0; u < 4; ++u) c[u] = (p + u < re) ? Bj[p + u] : 0x7fffffff;
                            int n = 0;
#pragma unroll
                            for (int u = 0; u < 4; ++u)
                                if (c[u] < hi) { set_bit(bits, (int)(c[u] - lo)); ++n; }
                            p += n;
                            if (n < 4) break;
                        }
                        seg_end[jj - nz0] = (uint32_t)(p - rb);
                    }
                }
                wsync();
                nnz_sw = popcount_prefix(bits, wpre, nw);
                if (nnz_sw <= G::CAP || nw == 1) break;
                nw = max(1, nw >> 1);   // too many entries for this window: halve it
            }
            for (int p = l; p < nnz_sw; p += WAVE) {
                acc[p] = (T)0;
                tag[p] = 0xffffffffu;
            }
            wsync();
            // ---- pass B: values, in (jj, kk) order, owner rounds for equal columns
            uint32_t seq = 0x3ffffffu;
            for (int64_t b = a0; b < a1; b += WAVE) {
                const int64_t jj = b + l;
                long long beg = 0;
                int cnt = 0;
                T av = (T)0;
                if (jj < a1) {
                    const int32_t k = Aj[jj];
                    av = Ax[jj];
                    const int64_t rb = Bp[k];
                    if (single) {
                        beg = rb;
                        cnt = (int)(Bp[k + 1] - rb);
                    } else {
                        const uint32_t cb = lo == 0 ? 0u : seg_cur[jj - nz0];
                        const uint32_t ce = seg_end[jj - nz0];
                        beg = rb + cb;
                        cnt = (int)(ce - cb);
                        seg_cur[jj - nz0] = ce;
                    }
                }
                for_each_product(beg, cnt, marker, [&](bool v, int s, long long idx) {
                    const T as = __shfl(av, s, WAVE);
                    int col = 0;
                    T bv = (T)0;
                    if (v) {
                        col = Bj[idx];
                        bv = Bx[idx];
                    }
                    const T prod = mul_rn(as, bv);
                    const int pos = v ? bit_pos(bits, wpre, (int)(col - lo)) : 0;
                    bool pending = v;
                    while (__ballot(pending)) {
                        if (seq == 0u) {   // tag space exhausted: re-arm (rare)
                            wsync();
                            for (int p = l; p < nnz_sw; p += WAVE) tag[p] = 0xffffffffu;
                            seq = 0x3ffffffu;
                            wsync();
                        }
                        const uint32_t key = (seq << 6) | (uint32_t)l;
                        if (pending) atomicMin(&tag[pos], key);
                        wsync();
                        if (pending && tag[pos] == key) {
                            acc[pos] = add_rn(acc[pos], prod);
                            pending = false;
                        }
                        wsync();
                        --seq;
                    }
                });
            }
            wsync();
            // ---- compress: column list in sorted order from the bitmap, then coalesced store
            for (int w = l; w < nw; w += WAVE) {
                uint32_t x = bits[w];
                uint32_t p = wpre[w];
                while (x) {
                    const int bb = __builtin_ctz(x);
                    tag[p++] = (uint32_t)(lo + 32 * w + bb);
                    x &= x - 1u;
                }
            }
            wsync();
            const int64_t o = out0 + written;
            for (int p = l; p < nnz_sw; p += WAVE) {
                Cj[o + p] = (int32_t)tag[p];
                Cx[o + p] = (alpha == (T)1) ? acc[p] : mul_rn(alpha, acc[p]);
            }
            written += nnz_sw;
            wsync();
            lo = hi;
        }
    }
    if (UB && l == 0) row_cnt[row] = written;
}

// ---------------------------------------------------------------------------------------
// ALG1 copy phase: move each row from its upper-bound slot to its final slot, scaling by
// alpha (cusparseSpGEMM_copy).  One wave per row.
template <typename T, typename IPC>
__global__ __launch_bounds__(BLOCK) void k_compact(int64_t rows, const int64_t* __restrict__ ub,
                                                   const IPC* __restrict__ Cp,
                                                   const int32_t* __restrict__ Tj,
                                                   const T* __restrict__ Tx,
                                                   int32_t* __restrict__ Cj, T* __restrict__ Cx,
                                                   T alpha) {
    const int l = lane_id();
    const int64_t row = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
    if (row >= rows) return;
    const int64_t s = ub[row];
    const int64_t d = (int64_t)Cp[row];
    const int64_t n = (int64_t)Cp[row + 1] - d;
    for (int64_t p = l; p < n; p += WAVE) {
        Cj[d + p] = Tj[s + p];
        const T x = Tx[s + p];
        Cx[d + p] = (alpha == (T)1) ? x : mul_rn(alpha, x);
    }
}

// ---------------------------------------------------------------------------------------
// Canonical-format / bounds check.  flags[0] |= order violation, flags[1] |= bad index or
// bad indptr.  One thread per row.
template <typename IP>
__global__ __launch_bounds__(BLOCK) void k_validate(int64_t rows, int64_t cols, int64_t nnz,
                                                    const IP* __restrict__ p,
                                                    const int32_t* __restrict__ j,
                                                    int* __restrict__ flags) {
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= rows) return;
    const int64_t p0 = p[i], p1 = p[i + 1];
    if (p0 < 0 || p1 < p0 || p1 > nnz) {
        atomicOr(&flags[1], 1);
        return;
    }
    int prev = -1;
    for (int64_t q = p0; q < p1; ++q) {
        const int c = j[q];
        if (c < 0 || c >= cols) atomicOr(&flags[1], 1);
        if (c <= prev) atomicOr(&flags[0], 1);
        prev = c;
    }
}

}  // namespace spg
