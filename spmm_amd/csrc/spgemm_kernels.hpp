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

// Total number of products P = sum over A's entries of the length of the B row they select
// (flat over A's entries, one atomic per block; `out` must be zero).
template <typename IP>
__global__ __launch_bounds__(BLOCK) void k_products_total(int64_t nnzA, const int32_t* __restrict__ Aj,
                                                          const IP* __restrict__ Bp,
                                                          unsigned long long* __restrict__ out) {
    __shared__ long long part[WPB];
    long long s = 0;
    const int64_t stride = (int64_t)gridDim.x * BLOCK;
    int64_t e = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    for (; e + 3 * stride < nnzA; e += 4 * stride) {   // four independent gathers in flight
        int32_t k[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) k[u] = Aj[e + u * stride];
#pragma unroll
        for (int u = 0; u < 4; ++u) s += (long long)(Bp[k[u] + 1] - Bp[k[u]]);
    }
    for (; e < nnzA; e += stride) {
        const int32_t k = Aj[e];
        s += (long long)(Bp[k + 1] - Bp[k]);
    }
    s = wave_sum64(s);
    if (lane_id() == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        long long t = 0;
        for (int w = 0; w < WPB; ++w) t += part[w];
        if (t) atomicAdd(out, (unsigned long long)t);
    }
}

// ---------------------------------------------------------------------------------------
// Symbolic phase (general path): structural nnz of each output row (no values).  One wave
// per row, a private bitmap window in LDS.  Rows of C wider than one window walk B with
// cursors.  Rows come either from the range [row0, row0 + nrows) or, when `list` is not
// null, from list[0 .. *list_count) (rows the short-row kernel spilled); waves loop over
// their share of rows.
template <typename IP>
__global__ __launch_bounds__(BLOCK) void k_symbolic(
    int64_t row0, int64_t nrows, int64_t ncols, const IP* __restrict__ Ap,
    const int32_t* __restrict__ Aj, const IP* __restrict__ Bp, const int32_t* __restrict__ Bj,
    int64_t* __restrict__ row_cnt, uint32_t* __restrict__ cur, int64_t nz0,
    const int32_t* __restrict__ list, const int32_t* __restrict__ list_count) {
    __shared__ uint32_t lds[WPB][SymGeom::BYTES / 4];
    const int l = lane_id();
    const int wv = threadIdx.x >> 6;
    uint32_t* bits = lds[wv];
    int* marker = (int*)(bits + SymGeom::NWMAX);
    const int64_t count = list ? (int64_t)*list_count : nrows;
    for (int64_t it = (int64_t)blockIdx.x * WPB + wv; it < count; it += (int64_t)gridDim.x * WPB) {
        const int64_t row = list ? (int64_t)list[it] : row0 + it;
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
    uint32_t* __restrict__ seg, int64_t nz0, int64_t seg_len, const int32_t* __restrict__ list,
    const int32_t* __restrict__ list_count) {
    using G = NumGeom<T>;
    __shared__ __attribute__((aligned(16))) char lds_raw[WPB][G::BYTES];
    const int l = lane_id();
    const int wv = threadIdx.x >> 6;
    const int64_t count = list ? (int64_t)*list_count : nrows;
    for (int64_t it = (int64_t)blockIdx.x * WPB + wv; it < count; it += (int64_t)gridDim.x * WPB) {
    const int64_t row = list ? (int64_t)list[it] : row0 + it;
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
                    const T as = shfl_v(av, s);
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
                        if (pending && __hip_atomic_load(&tag[pos], __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_WAVEFRONT) == key) {
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
    }  // rows of this wave
}

// ---------------------------------------------------------------------------------------
// Short-row kernel: one wave per output row whose A row has <= 64 entries, whose product
// count is <= PLONG, whose structural nnz is <= CAP and whose columns fit one 16384-column
// bitmap (the shape of BASELINE config 2).  Products are enumerated in flattened (jj, kk)
// order, 64 per step: a step's lanes find their A entry with a marker write + DPP max
// scan, so every product of the row is fetched with independent loads (one memory round
// trip when the row has <= 512 products: they stay in registers between the structure
// and the value pass; longer rows re-read B for the value pass).  The bitmap is kept as 8
// contiguous words per lane (b128 LDS access), its popcount prefix gives each column its
// output position, values are added in (jj, kk) order with lowest-lane-first owner rounds,
// and each lane writes its own run of the (already sorted) output.
// MODE: SHORT_SYM counts nnz per row (ALG2/3 symbolic), SHORT_NUM writes at C's exact row
// pointer, SHORT_NUMUB writes at an upper-bound offset and records nnz (ALG1).  Rows outside
// the limits are appended to `spill` (handled by the next kernel; the list order does not
// affect any result).  Rows come from [row0, row0 + nrows) or, with `list`, from
// list[0 .. *list_count).
// SHORT_NUMLB (ALG1 single pass): one wave per row, rows in dispatch order.  The rows of a
// block share one decoupled look-back (see lb_lead): each row gets its offset and writes its
// columns and values straight into Cj/Cx -- at most `cap` entries; a row past that sets
// scal[LB_CAPX] and writes nothing -- and its row pointer into Cp.  A row this kernel cannot
// take sets scal[LB_FAIL].  Either flag makes the host redo the product two-phase.
enum { SHORT_SYM = 0, SHORT_NUM = 1, SHORT_NUMUB = 2, SHORT_NUMLB = 3 };
enum { LB_TICKET = 6, LB_FAIL = 7, LB_TOTAL = 8, LB_OVERFLOW = 9, LB_CAPX = 10 };

// Block `row` publishes its aggregate (flag 1) or, for block 0, its inclusive prefix (flag 2).
__device__ __forceinline__ void lb_publish(unsigned long long* st, int64_t row, int64_t v, int l) {
    if (l == 0)
        __hip_atomic_store(&st[row], ((row == 0 ? 2ull : 1ull) << 62) | (unsigned long long)v,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Exclusive prefix of `row` by looking back over its predecessors 64 at a time; publishes
// the row's inclusive prefix.  Rows are mapped statically (row = wave id), so a wave may
// wait on a row whose wave has not been dispatched yet: the wait is bounded by LB_SPIN
// wall-clock ticks (100 MHz), after which the row sets `*fail` (the host then discards the
// pass) and carries on, so the grid always drains.
constexpr uint64_t LB_SPIN = 2000000;   // 20 ms
__device__ __forceinline__ int64_t lb_lookback(unsigned long long* st, int64_t row, int64_t v, int l,
                                               int64_t* fail) {
    constexpr unsigned long long VMASK = (1ull << 62) - 1;
    if (row == 0) return 0;
    long long prefix = 0;
    int64_t j = row - 1;
    const uint64_t t0 = wall_clock64();
    for (;;) {
        const int64_t q = j - l;
        unsigned long long s = 0;
        if (q >= 0) {
            do {
                s = __hip_atomic_load(&st[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((s >> 62) == 0 && wall_clock64() - t0 > LB_SPIN) {
                    *fail = 1;
                    s = 2ull << 62;   // give up: treat as an inclusive zero
                }
            } while ((s >> 62) == 0);
        }
        const unsigned long long incm = __ballot(q >= 0 && (s >> 62) == 2);
        const int stop = incm ? __ffsll((long long)incm) - 1 : WAVE;
        const long long val = (q >= 0 && l <= stop) ? (long long)(s & VMASK) : 0;
        prefix += wave_sum64(val);
        if (incm || j - WAVE < 0) break;
        j -= WAVE;
    }
    if (l == 0)
        __hip_atomic_store(&st[row], (2ull << 62) | (unsigned long long)(prefix + v), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    return prefix;
}

template <int CAP_, int PLONG_, int WPB_, int R_> struct ShortCfg {
    static constexpr int R = R_;               // register-resident products per lane
    static constexpr int PREG = R * WAVE;      // 512: rows up to this keep products in VGPRs
    static constexpr int PLONG = PLONG_;       // longest product list taken
    static constexpr int CAP = CAP_;           // most output entries per row
    static constexpr int NW = 512;             // bitmap words: <= 16384 columns
    static constexpr int WPB = WPB_;           // waves per block
    static constexpr int MKB = (PREG + 511) / 512 * 512;   // marker bytes (8 per lane per piece)
};
using ShortSmall = ShortCfg<320, 65535, 4, 8>;     // ~10 KB LDS per wave: 16 waves / CU;
                                                   // 640 products per row in registers

template <typename T, typename IP, typename G, bool VALS> struct ShortLds {
    uint32_t bits[G::NW];
    uint16_t wpre[G::NW];
    T acc[VALS ? G::CAP + 1 : 1];              // + a dummy slot; marker bytes in pass 1
    uint32_t tag[VALS ? G::CAP + 1 : 1];
    int8_t mk[VALS ? 1 : G::MKB];              // symbolic mode: its own marker bytes
    T ja[WAVE];
    IP jb0[WAVE];
    uint16_t joff[WAVE];
    int8_t marker[WAVE + 4];                   // + a dummy byte
};

// Lane -> A-entry map for the 64 products starting at c0: lanes whose segment starts in
// [c0, c0+64) drop their lane id at that offset, a DPP max-scan (seeded with the carry of
// the previous chunk) fills the gaps.  Branch-free: lanes with nothing to mark write the
// dummy byte.  Returns the A entry (lane) of product c0 + lane; updates `carry`.
template <typename L>
__device__ __forceinline__ int chunk_src(L& S, int l, int cnt, int off, int c0, int& carry) {
    S.marker[l] = -1;
    wsync();
    if (cnt > 0 && off >= c0 && off < c0 + WAVE) S.marker[off - c0] = (int8_t)l;
    wsync();
    const int src = max(wave_incl_max_dpp((int)S.marker[l]), carry);
    carry = readlane_i(src, WAVE - 1);
    return src;
}

template <typename T, typename IP, typename OFF, int MODE, typename G>
__global__ __launch_bounds__(G::WPB * WAVE, sizeof(T) <= 8 ? 5 : 2) void k_short(
    int64_t row0, int64_t nrows, int64_t ncols, const IP* __restrict__ Ap,
    const int32_t* __restrict__ Aj, const T* __restrict__ Ax, const IP* __restrict__ Bp,
    const int32_t* __restrict__ Bj, const T* __restrict__ Bx, const OFF* __restrict__ Coff,
    int32_t* __restrict__ Cj, T* __restrict__ Cx, T alpha, int64_t* __restrict__ row_cnt,
    int32_t* __restrict__ spill, int32_t* __restrict__ spill_count,
    const int32_t* __restrict__ list, const int32_t* __restrict__ list_count,
    unsigned long long* __restrict__ lb, OFF* __restrict__ Cp, int64_t* __restrict__ scal, int64_t cap) {
    constexpr int R = G::R;
    constexpr bool LB = MODE == SHORT_NUMLB;
    constexpr bool VALS = MODE != SHORT_SYM;
    __shared__ __attribute__((aligned(16))) ShortLds<T, IP, G, VALS> lds[G::WPB];
    const int l = lane_id();
    const int wv = uniform((int)(threadIdx.x >> 6));
    ShortLds<T, IP, G, VALS>& S = lds[wv];
    const int64_t count = list ? (int64_t)*list_count : nrows;
    // LB: a row with no entries (or one this kernel cannot take) still publishes and writes
    // its row pointer
    // LB: one look-back per block (its WPB consecutive rows, one per wave).  A wave drops
    // its row count in LDS and goes on; wave 0 waits for the WPB counts, publishes the
    // block's aggregate, looks back over earlier blocks and posts the block's base; a wave
    // waits for the base only when it is about to write.  Every wave arrives exactly once
    // (rows past the end with 0).
    __shared__ long long lb_v[G::WPB];
    __shared__ long long lb_base;
    __shared__ int lb_arrived, lb_ready;
    if (LB) {
        if (threadIdx.x == 0) {
            lb_arrived = 0;
            lb_ready = 0;
        }
        __syncthreads();
    }
    auto lb_arrive = [&](int64_t v) {
        if (l == 0) {
            lb_v[wv] = v;
            __hip_atomic_fetch_add(&lb_arrived, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    };
    auto lb_lead = [&]() {   // wave 0
        while (__hip_atomic_load(&lb_arrived, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < G::WPB)
            __builtin_amdgcn_s_sleep(1);
        long long agg = 0;
#pragma unroll
        for (int w = 0; w < G::WPB; ++w) agg += lb_v[w];
        lb_publish(lb, blockIdx.x, agg, l);
        const int64_t pre = lb_lookback(lb, blockIdx.x, agg, l, &scal[LB_FAIL]);
        if (l == 0) {
            lb_base = pre;
            __hip_atomic_store(&lb_ready, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    };
    auto lb_row_base = [&](int64_t row, int64_t v) -> int64_t {
        while (__hip_atomic_load(&lb_ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
            __builtin_amdgcn_s_sleep(1);
        long long pre = lb_base;
        for (int w = 0; w < wv; ++w) pre += lb_v[w];
        if (l == 0) {
            Cp[row] = (OFF)pre;
            if (row == nrows - 1) {
                const int64_t tot = pre + v;
                Cp[nrows] = (OFF)tot;
                scal[LB_TOTAL] = tot;
                scal[LB_OVERFLOW] = (sizeof(OFF) == 4 && tot > 2147483647LL) ? 1 : 0;
            }
        }
        return pre;
    };
    auto lb_block = [&](int64_t row, int64_t v) -> int64_t {
        lb_arrive(v);
        if (wv == 0) lb_lead();
        return lb_row_base(row, v);
    };
    auto lb_empty = [&](int64_t row, bool fail) {
        if (l == 0) {
            if (fail) scal[LB_FAIL] = 1;
            row_cnt[row] = 0;
        }
        lb_block(row, 0);
    };
    auto process = [&](int64_t it) {
        const int64_t row = list ? (int64_t)uniform(list[it]) : row0 + it;
        const int64_t a0 = Ap[row];
        const int nA = (int)(Ap[row + 1] - a0);
        if (nA <= 0 || ncols <= 0) {
            if (LB) lb_empty(row, false);
            else if (MODE != SHORT_NUM && l == 0) row_cnt[row] = 0;
            return;
        }
        if (nA > WAVE || ncols > 32LL * G::NW) {
            if (LB) lb_empty(row, true);
            else if (l == 0) spill[atomicAdd(spill_count, 1)] = (int32_t)row;
            return;
        }
        int cnt = 0;
        IP b0 = 0;
        T av = (T)0;
        if (l < nA) {
            const int32_t k = Aj[a0 + l];
            b0 = Bp[k];
            cnt = (int)(Bp[k + 1] - b0);
            if (VALS) av = Ax[a0 + l];
        }
        const int incl = wave_incl_sum_dpp(cnt);
        const int off = incl - cnt;
        const int P = readlane_i(incl, WAVE - 1);
        if (P > G::PLONG) {
            if (LB) lb_empty(row, true);
            else if (l == 0) spill[atomicAdd(spill_count, 1)] = (int32_t)row;
            return;
        }
        if (P == 0) {
            if (LB) lb_empty(row, false);
            else if (MODE != SHORT_NUM && l == 0) row_cnt[row] = 0;
            return;
        }
        S.jb0[l] = b0;
        S.joff[l] = (uint16_t)off;
        if (VALS) S.ja[l] = av;
        uint4* bits4 = reinterpret_cast<uint4*>(S.bits);
        bits4[2 * l] = make_uint4(0u, 0u, 0u, 0u);
        bits4[2 * l + 1] = make_uint4(0u, 0u, 0u, 0u);
        wsync();
        const int nch = (P + WAVE - 1) / WAVE;
        const bool inreg = P <= G::PREG;
        int col[R];
        T prd[R];
        int carry = -1;
        // ---- pass 1: structure; for short lists the products stay in registers
        if (inreg) {
            // lane -> A-entry map of every chunk at once: each A entry drops its lane id at
            // the first product it owns, a DPP max-scan per chunk (carried across chunks)
            // fills the gaps.  The marker bytes borrow the accumulator area.
            int8_t* mk = VALS ? reinterpret_cast<int8_t*>(S.acc) : S.mk;
            static_assert(!VALS || G::MKB <= (int)sizeof(T) * G::CAP, "markers must fit acc");
#pragma unroll
            for (int q = 0; q < G::MKB / (WAVE * 8); ++q)
                reinterpret_cast<uint64_t*>(mk)[q * WAVE + l] = ~0ull;
            wsync();
            if (cnt > 0) mk[off] = (int8_t)l;
            wsync();
            int mrk[R];
#pragma unroll
            for (int r = 0; r < R; ++r) mrk[r] = r < nch ? (int)mk[r * WAVE + l] : -1;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                col[r] = -1;
                prd[r] = (T)0;
                if (r < nch) {
                    const int src = max(wave_incl_max_dpp(mrk[r]), carry);
                    carry = readlane_i(src, WAVE - 1);
                    const int t = r * WAVE + l;
                    const bool v = t < P;
                    const IP idx = v ? S.jb0[src] + (IP)(t - (int)S.joff[src]) : (IP)0;
                    const int c = Bj[idx];
                    if (VALS) prd[r] = mul_rn(S.ja[src], Bx[idx]);
                    col[r] = v ? c : -1;
                    if (v) set_bit(S.bits, c);
                }
            }
        } else {
            for (int c0 = 0; c0 < P; c0 += WAVE) {
                const int src = chunk_src(S, l, cnt, off, c0, carry);
                const int t = c0 + l;
                const bool v = t < P;
                const IP idx = v ? S.jb0[src] + (IP)(t - (int)S.joff[src]) : (IP)0;
                const int c = Bj[idx];
                if (v) set_bit(S.bits, c);
            }
        }
        wsync();
        // ---- popcount prefix over this lane's 8 contiguous words
        const uint4 q0 = bits4[2 * l], q1 = bits4[2 * l + 1];
        const int c0 = __popc(q0.x), c1 = __popc(q0.y), c2 = __popc(q0.z), c3 = __popc(q0.w);
        const int c4 = __popc(q1.x), c5 = __popc(q1.y), c6 = __popc(q1.z), c7 = __popc(q1.w);
        const int mine = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
        const int pincl = wave_incl_sum_dpp(mine);
        const int nnz = readlane_i(pincl, WAVE - 1);
        if (MODE == SHORT_SYM) {
            if (l == 0) row_cnt[row] = nnz;
            return;
        }
        // LB: publish, then look back at once -- an inclusive prefix published promptly is
        // what keeps successors' look-backs short
        int64_t cbase = -1;
        if (LB) {
            lb_arrive(nnz);
            if (wv == 0) lb_lead();
        }
        const int p0 = pincl - mine;
        {
            const int p1 = p0 + c0, p2 = p1 + c1, p3 = p2 + c2, p4 = p3 + c3, p5 = p4 + c4,
                      p6 = p5 + c5, p7 = p6 + c6;
            uint4 w;
            w.x = (uint32_t)p0 | ((uint32_t)p1 << 16);
            w.y = (uint32_t)p2 | ((uint32_t)p3 << 16);
            w.z = (uint32_t)p4 | ((uint32_t)p5 << 16);
            w.w = (uint32_t)p6 | ((uint32_t)p7 << 16);
            reinterpret_cast<uint4*>(S.wpre)[l] = w;
        }
        // ---- pass 2: values in (jj, kk) order; equal columns of one step go lowest lane
        // first (ds_min on an owner tag).  `wb` is the first output position of the column
        // window being accumulated (0 for rows that fit CAP).
        uint32_t seq = 0x3ffffffu;
        auto accumulate = [&](int c, T pv, int wb) -> int {
            int pos = G::CAP;
            if (c >= 0) {
                const int w = c >> 5;
                pos = (int)S.wpre[w] + __popc(S.bits[w] & ((1u << (c & 31)) - 1u)) - wb;
            }
            bool pending = c >= 0;
            // (no fences inside: the atomic and the atomic load of one address keep their
            // order, and LDS operations of a wave execute in issue order)
            while (__ballot(pending)) {
                const uint32_t key = (seq << 6) | (uint32_t)l;
                if (pending) {
                    atomicMin(&S.tag[pos], key);
                    if (__hip_atomic_load(&S.tag[pos], __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WAVEFRONT) == key) {
                        S.acc[pos] = add_rn(S.acc[pos], pv);
                        pending = false;
                    }
                }
                --seq;
            }
            return pos;
        };
        // Column windows made of whole lanes' 8-word groups (<= 256 entries each, so a
        // window always advances), each holding <= CAP entries; rows with nnz <= CAP are one
        // window.  Register-resident products are filtered per window; longer rows re-read
        // the window's products from B (L2-resident by now).
        for (int L0 = 0; L0 < WAVE;) {
            int L1 = WAVE, wb = 0, wn = nnz;
            if (nnz > G::CAP) {
                wb = readlane_i(p0, L0);
                L1 = (int)__popcll(__ballot(pincl <= wb + G::CAP));
                if (L1 <= L0) L1 = L0 + 1;
                wn = (L1 < WAVE ? readlane_i(p0, L1) : nnz) - wb;
            }
            const int clo = 256 * L0, chi = 256 * L1;
            for (int p = l; p < wn; p += WAVE) {
                S.acc[p] = (T)0;
                S.tag[p] = 0xffffffffu;
            }
            wsync();
            seq = 0x3ffffffu;
            if (inreg) {
                int pos[R];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    pos[r] = G::CAP;
                    if (r < nch)
                        pos[r] = accumulate(col[r] >= clo && col[r] < chi ? col[r] : -1, prd[r], wb);
                }
                wsync();
                // column list straight from the registers (equal columns write equal values)
#pragma unroll
                for (int r = 0; r < R; ++r)
                    if (r < nch && pos[r] < G::CAP) S.tag[pos[r]] = (uint32_t)col[r];
            } else {
                carry = -1;
                for (int cc0 = 0; cc0 < P; cc0 += WAVE) {
                    const int src = chunk_src(S, l, cnt, off, cc0, carry);
                    const int t = cc0 + l;
                    const bool v = t < P;
                    const IP idx = v ? S.jb0[src] + (IP)(t - (int)S.joff[src]) : (IP)0;
                    const int c = Bj[idx];
                    const T pv = mul_rn(S.ja[src], Bx[idx]);
                    accumulate(v && c >= clo && c < chi ? c : -1, pv, wb);
                    if (seq < 4096u) {   // re-arm the tag space (very long rows only)
                        wsync();
                        for (int p = l; p < wn; p += WAVE) S.tag[p] = 0xffffffffu;
                        seq = 0x3ffffffu;
                        wsync();
                    }
                }
                wsync();
                if (l >= L0 && l < L1) {   // column list from this lane's 8 bitmap words
                    uint64_t m0 = (uint64_t)q0.x | ((uint64_t)q0.y << 32);
                    uint64_t m1 = (uint64_t)q0.z | ((uint64_t)q0.w << 32);
                    uint64_t m2 = (uint64_t)q1.x | ((uint64_t)q1.y << 32);
                    uint64_t m3 = (uint64_t)q1.z | ((uint64_t)q1.w << 32);
                    const int cbase = 256 * l;
                    int p = p0 - wb;
                    while (m0 | m1 | m2 | m3) {
                        int cc;
                        if (m0) { cc = cbase + __builtin_ctzll(m0); m0 &= m0 - 1; }
                        else if (m1) { cc = cbase + 64 + __builtin_ctzll(m1); m1 &= m1 - 1; }
                        else if (m2) { cc = cbase + 128 + __builtin_ctzll(m2); m2 &= m2 - 1; }
                        else { cc = cbase + 192 + __builtin_ctzll(m3); m3 &= m3 - 1; }
                        S.tag[p++] = (uint32_t)cc;
                    }
                }
            }
            wsync();
            if (LB && cbase < 0) {
                cbase = lb_row_base(row, nnz);
                if (cbase + nnz > cap && l == 0) scal[LB_CAPX] = 1;   // output buffer too small
            }
            const int64_t rbase = LB ? cbase : (int64_t)Coff[row];
            int32_t* __restrict__ crow = Cj + rbase + wb;
            T* __restrict__ xrow = Cx + rbase + wb;
            const int wlim = (LB && cbase + nnz > cap) ? 0 : wn;
            for (int p = l; p < wlim; p += WAVE) {
                crow[p] = (int32_t)S.tag[p];
                const T val = S.acc[p];
                xrow[p] = (alpha == (T)1) ? val : mul_rn(alpha, val);
            }
            wsync();
            L0 = L1;
        }
        if ((MODE == SHORT_NUMUB || LB) && l == 0) row_cnt[row] = nnz;
        wsync();
    };
    // (LB: the grid has one wave per row, so every wave meets lb_block exactly once)
    for (int64_t it = (int64_t)blockIdx.x * G::WPB + wv; it < count; it += (int64_t)gridDim.x * G::WPB)
        process(it);
    if (LB && (int64_t)blockIdx.x * G::WPB + wv >= count) lb_arrive(0);
}

// ---------------------------------------------------------------------------------------
// Single-pass exclusive scan with decoupled look-back.  out[0..n) = exclusive prefix of
// in[] (plus *seed when given), out[n] = total, scalars[0] = total, scalars[1] = 1 if the
// total overflows OUT.
// `status` holds 1 ticket word + one 8-byte status per tile and must be zero on entry.
// Status word: bits 63..62 = 0 not ready / 1 tile aggregate / 2 inclusive prefix,
// bits 61..0 = value.  Tiles take tickets in order, so every tile a block waits on has
// started; the status word is its own payload (8-byte agent-scope atomics on both sides,
// MI355X_MICROARCH.md, "Valid forms").
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = BLOCK * SCAN_ITEMS;   // 2048
// word of the host-pinned buffer that carries the generation of the last mirrored scan (past
// every word read_scalars fills)
constexpr int MIRROR_GEN_WORD = 16 + 1024;

constexpr unsigned long long SCAN_VMASK = (1ull << 62) - 1;
constexpr unsigned long long GPRE_READY = 1ull << 63;

// LDS of one scan tile (a block of BLOCK threads)
struct ScanLds {
    long long wsum[WPB];
    long long prefix;
};

// One tile of the scan, tile index `bid` (tiles below it have started).  `st` = the tile
// status words (status + 1).  With `gpre`, the exclusive prefix at every 64-element group
// start also goes to gpre[group] | GPRE_READY (agent-scope stores: k_row's ALG1 numeric
// pass reads its rows' offsets from them while the scan runs beside it).
// Bounded waits: a look-back that finds a predecessor's status word still
// empty after SCAN_SPIN wall-clock ticks (100 MHz: 2 ms) stops waiting and computes what it
// waited for directly from the inputs -- the exclusive prefix is the sum of in[0 .. base),
// all of which are in memory before the launch -- so the result is the same and the grid
// drains even if a predecessor tile were never scheduled (a dispatch order the ticket
// scheme already rules out).  The same bound guards k_row's wait on the 64-row group words.
constexpr uint64_t SCAN_SPIN = 200000;

// sum of in[0 .. n) over one wave (the fallback of a timed-out wait; never the fast path)
template <typename IN>
__device__ __forceinline__ long long wave_direct_sum(const IN* in, int64_t n) {
    long long s = 0;
    for (int64_t i = lane_id(); i < n; i += WAVE) s += (long long)in[i];
    return wave_sum64(s);
}

template <typename OUT, typename IN>
__device__ __forceinline__ void scan_tile(int64_t bid, int64_t n, const IN* in, OUT* out,
                                          unsigned long long* __restrict__ st, int64_t* __restrict__ scalars,
                                          int32_t* __restrict__ move_cnt, int64_t* __restrict__ move_dst,
                                          int64_t* __restrict__ host_mirror, int64_t mirror_gen, int mirror_n,
                                          const int64_t* seed, ScanLds& L,
                                          unsigned long long* __restrict__ gpre = nullptr,
                                          uint64_t spin = SCAN_SPIN) {
    static_assert(SCAN_ITEMS * 8 == WAVE, "8 threads per 64-element group");
    constexpr unsigned long long VMASK = SCAN_VMASK;
    long long* wsum = L.wsum;
    long long& prefix_s = L.prefix;
    const int tid = threadIdx.x, l = lane_id(), wv = tid >> 6;
    const int64_t base = bid * SCAN_TILE + (int64_t)tid * SCAN_ITEMS;
    long long v[SCAN_ITEMS];
    long long tsum = 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        v[j] = base + j < n ? in[base + j] : 0;
        tsum += v[j];
    }
    const long long incl = wave_incl_sum64(tsum);
    if (l == WAVE - 1) wsum[wv] = incl;
    __syncthreads();
    long long wbase = 0, btot = 0;
#pragma unroll
    for (int q = 0; q < WPB; ++q) {
        if (q < wv) wbase += wsum[q];
        btot += wsum[q];
    }
    if (wv == 0) {
        long long prefix = 0;
        if (bid == 0) {
            if (seed) prefix = *seed;   // a chunked scan continues from the previous chunk's total
            if (l == 0)
                __hip_atomic_store(&st[0], (2ull << 62) | (unsigned long long)(prefix + btot), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (l == 0)
                __hip_atomic_store(&st[bid], (1ull << 62) | (unsigned long long)btot, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            int64_t j = bid - 1;
            uint64_t t0 = 0;   // (the clock is read only once a predecessor is found not ready)
            bool late = spin == 0;   // (spin 0: the direct path, for the tests)
            for (; !late;) {
                const int64_t q = j - l;
                unsigned long long s = 0;
                if (q >= 0) {
                    do {
                        s = __hip_atomic_load(&st[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if ((s >> 62) == 0) {
                            const uint64_t now = wall_clock64();
                            if (t0 == 0) {
                                t0 = now;
                            } else if (now - t0 > spin) {
                                s = 2ull << 62;   // stop waiting (the direct sum below replaces the prefix)
                                late = true;
                            }
                        }
                    } while ((s >> 62) == 0);
                }
                if (__ballot(late)) break;
                const unsigned long long incm = __ballot(q >= 0 && (s >> 62) == 2);
                const int stop = incm ? __ffsll((long long)incm) - 1 : WAVE;
                const long long val = (q >= 0 && l <= stop) ? (long long)(s & VMASK) : 0;
                prefix += wave_sum64(val);
                if (incm || j - WAVE < 0) break;
                j -= WAVE;
            }
            if (__ballot(late)) prefix = (seed ? *seed : 0) + wave_direct_sum(in, bid * SCAN_TILE);
            if (l == 0)
                __hip_atomic_store(&st[bid], (2ull << 62) | (unsigned long long)(prefix + btot),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (l == 0) prefix_s = prefix;
    }
    __syncthreads();
    long long run = prefix_s + wbase + incl - tsum;
    if (gpre && (tid & 7) == 0 && base < n)
        __hip_atomic_store(&gpre[base >> 6], GPRE_READY | (unsigned long long)run, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        if (base + j < n) out[base + j] = (OUT)run;
        run += v[j];
    }
    const int64_t ntiles = n > 0 ? (n + SCAN_TILE - 1) / SCAN_TILE : 1;
    if (bid != ntiles - 1) return;
    if (tid == 0) {
        const long long total = prefix_s + btot;
        out[n] = (OUT)total;
        const int64_t ovf = (sizeof(OUT) == 4 && total > 2147483647LL) ? 1 : 0;
        scalars[0] = total;
        scalars[1] = ovf;
        int64_t moved = 0;
        if (move_cnt) {   // (ALG1 on k_row) hand the spill count over (to scalars[5]) and re-arm
            moved = *move_cnt;
            *move_dst = moved;
            *move_cnt = 0;
        }
        // the control scalars (total, overflow, the symbolic pass's words, then the chunks'
        // spill counts) to pinned host memory, one thread, 16 independent loads at a time (a
        // block-wide system fence costs more than the few words a call has)
        if (mirror_n > 0) {
            __hip_atomic_store(&host_mirror[0], (int64_t)total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&host_mirror[1], ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (move_cnt) __hip_atomic_store(&host_mirror[5], moved, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        for (int b = 2; b < mirror_n; b += 16) {
            int64_t w[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) w[i] = b + i < mirror_n ? scalars[b + i] : 0;
#pragma unroll
            for (int i = 0; i < 16; ++i)
                if (b + i < mirror_n)
                    __hip_atomic_store(&host_mirror[b + i], w[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        // the call's generation last: the host polls it instead of waiting for the stream
        if (mirror_n > 0)
            __hip_atomic_store(&host_mirror[MIRROR_GEN_WORD], mirror_gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <typename OUT, typename IN = int64_t>
__global__ __launch_bounds__(BLOCK) void k_scan_lb(int64_t n, const IN* in, OUT* out,
                                                   unsigned long long* __restrict__ status,
                                                   int64_t* __restrict__ scalars,
                                                   int32_t* __restrict__ move_cnt = nullptr,
                                                   int64_t* __restrict__ move_dst = nullptr,
                                                   int64_t* __restrict__ host_mirror = nullptr,
                                                   int64_t mirror_gen = 0, int mirror_n = 0,
                                                   const int64_t* seed = nullptr, uint64_t spin = SCAN_SPIN) {
    __shared__ ScanLds L;
    __shared__ int bid_s;
    if (threadIdx.x == 0) bid_s = (int)atomicAdd(&status[0], 1ull);
    __syncthreads();
    // An in-place scan (the tile path's segment table and item counts) must not take the
    // bounded wait's direct-sum fallback: earlier tiles have already replaced their inputs
    // with exclusive prefixes, so in[0 .. base) no longer holds the counts.  Its
    // waits stay unbounded; the ticket order guarantees every predecessor has started.
    const bool in_place = reinterpret_cast<const void*>(in) == reinterpret_cast<const void*>(out);
    scan_tile<OUT, IN>(bid_s, n, in, out, status + 1, scalars, move_cnt, move_dst, host_mirror, mirror_gen,
                       mirror_n, seed, L, nullptr, in_place ? ~0ull : spin);
}

// ---------------------------------------------------------------------------------------
// ALG1 single pass, numeric call: C from the compact arrays in the workspace, scaled by
// alpha (in place when C points into the workspace).
template <typename T>
__global__ __launch_bounds__(BLOCK) void k_copy_scale(int64_t n, const int32_t* __restrict__ sj,
                                                      const T* __restrict__ sx, int32_t* __restrict__ dj,
                                                      T* __restrict__ dx, T alpha) {
    const bool copy_j = dj != sj;
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLOCK) {
        if (copy_j) dj[i] = sj[i];
        const T v = sx[i];
        dx[i] = alpha == (T)1 ? v : mul_rn(alpha, v);
    }
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
