// spgemm_row.hpp -- the short-row kernel (one wave per output row) for C rows of the shape
// of BASELINE config 2: A rows of <= 64 entries, <= PREG products, C <= 16384 columns.
//
// Same arithmetic as every other path (scipy csr_matmat order, see spg_device.hpp); what
// differs is how the order is kept cheaply.  Per row:
//
//   pass 1  every product of the row is fetched once into registers (PREG = R*64 of them),
//           its column set in an LDS bitmap with a returning ds_or.  A product whose bit was
//           already set marks its bitmap WORD as "duplicate" (dupw, one bit per word).
//   scan    popcount prefix over the bitmap -> each column's sorted output position; the
//           word's duplicate flag is folded into bit 15 of its prefix.
//   pass 2  a product in an unflagged word is the only contributor of its column: its value
//           is final (0 + a*b, scipy's sum starts at 0) and it is written straight from
//           registers to C at (row base + position).  Products in flagged words (typically
//           ~3 % of them) are compacted, in product order, into a list of <= LCAP entries;
//           lane i of the list sums, in list order, every entry of its position if it is
//           the first one (readlane loop, no atomics), and writes that column.
//
// So no product waits on another product: the LDS owner rounds of k_short (which order
// every accumulate) are gone from the common case.  Rows the kernel cannot take (> 64 A
// entries, > PREG products, > LCAP products in flagged words) are spilled -- by the same
// predicate in every mode, so the symbolic and numeric passes spill the same rows -- to the
// general kernel (k_symbolic / k_numeric over the spill list).
//
// MODES: ROW_SYM counts (ALG2/3 symbolic), ROW_NUM writes at C's row pointer (ALG2/3
// numeric), ROW_LB is the ALG1 single pass: every row publishes its count into a 64-ary
// arrival tree (LbTree), reads the exclusive prefix of its row from at most 4 tree levels
// (one load per lane per level, all issued before pass 2), and writes C's row pointer,
// columns and values in one launch.  Spilled rows still publish their count (the count-only
// loop below) and get their values from a k_numeric launch over the spill list afterwards.
#pragma once

#include "spgemm_kernels.hpp"

namespace spg {

enum { ROW_SYM = 0, ROW_NUM = 1, ROW_LB = 2 };

template <int R_, int LCAP_, int WPB_> struct RowCfg {
    static constexpr int R = R_;                     // register chunks of 64 products
    static constexpr int PREG = R * WAVE;            // most products a row may have
    static constexpr int LCAP = LCAP_;               // products in flagged words (<= WAVE)
    static constexpr int NW = 512;                   // bitmap words: <= 16384 columns
    static constexpr int WPB = WPB_;                 // waves per block
    static constexpr int MKB = (PREG + 511) / 512 * 512;   // marker bytes
    static_assert(LCAP <= WAVE, "one list entry per lane");
};
using RowSmall = RowCfg<10, 64, 4>;

template <typename T, typename IP, typename G, bool VALS> struct RowLds {
    uint32_t bits[G::NW];
    uint16_t wpre[G::NW];          // exclusive popcount prefix | 0x8000 for flagged words
    uint32_t dupw[G::NW / 32];     // one bit per bitmap word: a column of it was hit twice
    int8_t mk[G::MKB];             // lane -> A-entry markers of every chunk
    IP jb0[WAVE];                  // B row start of each A entry
    int32_t joff[WAVE];            // first flattened product of each A entry
    T ja[VALS ? WAVE : 1];         // A values
    T lx[VALS ? G::LCAP : 1];      // flagged-word products, in product order
    int32_t lc[VALS ? G::LCAP : 1];
    int32_t lp[VALS ? G::LCAP : 1];
    int8_t marker[WAVE + 4];       // count-only loop (one chunk at a time)
};

// ---- 64-ary arrival tree (ALG1 single pass) ------------------------------------------
// Level 0 has one unit per row; a level-(l+1) unit is a group of 64 consecutive level-l
// units.  agg[l][u] = READY | (sum of the counts under unit u).  grp[l][g] (l >= 1) counts
// arrivals of group g's level-(l-1) units in bits 57..63 and sums their values in bits
// 0..56: the unit whose arrival completes the group learns the group total from the value
// its add returns and publishes agg[l][g] (then arrives one level up).  A row's exclusive
// prefix is the sum, over every level, of the aggregates of the units that precede its own
// unit inside their group -- at most 63 words per level, one load per lane per level.
// No word is ever read before it is marked ready, so no fences are needed: every word is
// an 8-byte agent-scope atomic (MI355X_MICROARCH.md, "Valid forms": 8-B agent atomics on
// both sides).  Bounded by LB_SPIN like the block look-back.
struct LbTree {
    unsigned long long* agg[4];
    unsigned long long* grp[4];   // grp[0] unused
    long long n[4];               // units per level
    int top;                      // highest level (n[top] <= 64)
    unsigned long long* trace;    // optional: 4 wall-clock stamps per row (SPG_LB_TRACE)
};

constexpr unsigned long long LBT_READY = 1ull << 62;
constexpr unsigned long long LBT_VMASK = LBT_READY - 1;
constexpr unsigned long long LBT_ARRIVE = 1ull << 57;
constexpr unsigned long long LBT_SMASK = LBT_ARRIVE - 1;

__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Publish unit u of level lv with value v and arrive at its group; returns the value the
// arrival's add returned (lane 0), or ~0 when lv is the top level (no group).
__device__ __forceinline__ unsigned long long lbt_arrive(const LbTree& t, int lv, int64_t u, int64_t v, int l) {
    unsigned long long old = ~0ull;
    if (l == 0) {
        st_agent(&t.agg[lv][u], LBT_READY | (unsigned long long)v);
        if (lv < t.top)
            old = __hip_atomic_fetch_add(&t.grp[lv + 1][u >> 6], LBT_ARRIVE | (unsigned long long)v,
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return old;
}

// After an arrival at level lv: if it completed its group, publish the group and go on up.
__device__ __forceinline__ void lbt_cascade(const LbTree& t, int lv, int64_t u, int64_t v,
                                            unsigned long long old, int l) {
    for (;;) {
        if (lv >= t.top) return;
        const int64_t g = u >> 6;
        const long long size = min(64LL, t.n[lv] - (g << 6));
        const unsigned long long o0 = __builtin_amdgcn_readfirstlane((unsigned)(old & 0xffffffffu)) |
                                      ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(old >> 32)) << 32);
        if ((long long)(o0 >> 57) + 1 != size) return;   // not the last arrival
        v = (int64_t)(o0 & LBT_SMASK) + v;
        ++lv;
        u = g;
        old = lbt_arrive(t, lv, u, v, l);
    }
}

// Issue the loads of the row's prefix words (lane l of level lv: the l-th unit before the
// row's own unit in its group).  Lanes with nothing to read hold READY | 0.
__device__ __forceinline__ void lbt_issue(const LbTree& t, int64_t row, int l, unsigned long long s[4]) {
#pragma unroll
    for (int lv = 0; lv < 4; ++lv) {
        s[lv] = LBT_READY;
        if (lv <= t.top) {
            const int64_t u = row >> (6 * lv);
            const int idx = (int)(u & 63);
            if (l < idx) s[lv] = ld_agent(&t.agg[lv][u - idx + l]);
        }
    }
}

__device__ __forceinline__ int64_t lbt_wait(const LbTree& t, int64_t row, int l, unsigned long long s[4],
                                            int64_t* fail) {
    const uint64_t t0 = wall_clock64();
    for (;;) {
        bool nr = false;
#pragma unroll
        for (int lv = 0; lv < 4; ++lv) nr |= !(s[lv] & LBT_READY);
        if (!__ballot(nr)) break;
        if (wall_clock64() - t0 > LB_SPIN) {   // give up (the host redoes the product)
            if (l == 0) *fail = 1;
#pragma unroll
            for (int lv = 0; lv < 4; ++lv)
                if (!(s[lv] & LBT_READY)) s[lv] = LBT_READY;
            break;
        }
        __builtin_amdgcn_s_sleep(2);
#pragma unroll
        for (int lv = 0; lv < 4; ++lv) {
            if (!(s[lv] & LBT_READY)) {
                const int64_t u = row >> (6 * lv);
                s[lv] = ld_agent(&t.agg[lv][u - (int64_t)(u & 63) + l]);
            }
        }
    }
    long long sum = 0;
#pragma unroll
    for (int lv = 0; lv < 4; ++lv) sum += (long long)(s[lv] & LBT_VMASK);
    return wave_sum64(sum);
}

// Value of any of the four types from lane j (j wave-uniform).
template <typename T> __device__ __forceinline__ T readlane_v(T v, int j) {
    static_assert(sizeof(T) % 4 == 0, "32-bit parts");
    uint32_t w[sizeof(T) / 4];
    __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); ++i) w[i] = __builtin_amdgcn_readlane(w[i], j);
    T r;
    __builtin_memcpy(&r, w, sizeof(T));
    return r;
}

__device__ __forceinline__ int lane_rank(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

template <typename T> __device__ __forceinline__ T scale(T alpha, T v) {
    return alpha == (T)1 ? v : mul_rn(alpha, v);
}


template <int N> using IntC = std::integral_constant<int, N>;

// p[i]: a 32-bit byte offset from the (scalar) base when the index type is 32-bit, so the
// load takes the saddr form (one VGPR of address per load instead of two)
template <typename V, typename I> __device__ __forceinline__ V ld_idx(const V* __restrict__ p, I i) {
    if constexpr (sizeof(I) == 4) {
        const uint32_t o = (uint32_t)i * (uint32_t)sizeof(V);
        return *reinterpret_cast<const V*>(reinterpret_cast<const char*>(p) + (uint64_t)o);
    } else {
        return p[i];
    }
}

template <typename T, typename IP, typename OFF, int MODE, typename G>
__global__ __launch_bounds__(G::WPB * WAVE) void k_row(
    int64_t row0, int64_t nrows, int64_t ncols, const IP* __restrict__ Ap,
    const int32_t* __restrict__ Aj, const T* __restrict__ Ax, const IP* __restrict__ Bp,
    const int32_t* __restrict__ Bj, const T* __restrict__ Bx, const OFF* __restrict__ Coff,
    int32_t* __restrict__ Cj, T* __restrict__ Cx, T alpha, int64_t* __restrict__ row_cnt,
    int32_t* __restrict__ spill, int32_t* __restrict__ spill_count, LbTree tree,
    OFF* __restrict__ Cp, int64_t* __restrict__ scal, int64_t cap) {
    constexpr bool VALS = MODE != ROW_SYM;
    constexpr bool LB = MODE == ROW_LB;
    __shared__ __attribute__((aligned(16))) RowLds<T, IP, G, VALS> lds[G::WPB];
    const int l = lane_id();
    const int wv = uniform((int)(threadIdx.x >> 6));
    RowLds<T, IP, G, VALS>& S = lds[wv];
    const int64_t it = (int64_t)blockIdx.x * G::WPB + wv;
    if (it >= nrows) return;
    const int64_t row = row0 + it;
    uint4* bits4 = reinterpret_cast<uint4*>(S.bits);
    if (LB && tree.trace && l == 0) tree.trace[4 * row] = wall_clock64();

    // ---- LB: publish a count, then (after the value work) the row's base
    unsigned long long lbs[4];
    unsigned long long arrived = 0;
    auto lb_publish = [&](int64_t nnz) {
        if (tree.trace && l == 0) tree.trace[4 * row + 1] = wall_clock64();
        arrived = lbt_arrive(tree, 0, row, nnz, l);
        lbt_issue(tree, row, l, lbs);
        lbt_cascade(tree, 0, row, nnz, arrived, l);   // a completed group goes up at once
    };
    auto lb_base = [&](int64_t nnz) -> int64_t {   // -1: the output buffer is too small
        if (tree.trace && l == 0) tree.trace[4 * row + 2] = wall_clock64();
        const int64_t base = lbt_wait(tree, row, l, lbs, &scal[LB_FAIL]);
        if (tree.trace && l == 0) tree.trace[4 * row + 3] = wall_clock64();
        if (l == 0) {
            row_cnt[row] = nnz;   // a repeated spg_symbolic rescans the counts
            Cp[row] = (OFF)base;
            if (it == nrows - 1) {
                const int64_t tot = base + nnz;
                Cp[nrows] = (OFF)tot;
                scal[LB_TOTAL] = tot;
                scal[LB_OVERFLOW] = (sizeof(OFF) == 4 && tot > 2147483647LL) ? 1 : 0;
            }
            if (base + nnz > cap) scal[LB_CAPX] = 1;
        }
        return base + nnz > cap ? -1 : base;
    };
    auto spill_row = [&]() {
        if (l == 0) spill[atomicAdd(spill_count, 1)] = (int32_t)row;
    };

    const int64_t a0 = Ap[row];
    const int nA = (int)(Ap[row + 1] - a0);
    int cnt = 0, off = 0, P = 0;
    bool fits = nA > 0 && nA <= WAVE && ncols > 0;
    if (fits) {
        IP b0 = 0;
        T av = (T)0;
        if (l < nA) {
            const int32_t k = Aj[a0 + l];
            b0 = Bp[k];
            cnt = (int)(Bp[k + 1] - b0);
            if (VALS) av = Ax[a0 + l];
        }
        const int incl = wave_incl_sum_dpp(cnt);
        off = incl - cnt;
        P = readlane_i(incl, WAVE - 1);
        S.jb0[l] = b0;
        S.joff[l] = off;
        if (VALS) S.ja[l] = av;
        fits = P <= G::PREG;
    }

    // ---- the register path: NC chunks of 64 products, straight-line
    auto row_body = [&](auto nct) {
        constexpr int NC = decltype(nct)::value;
        bits4[2 * l] = make_uint4(0u, 0u, 0u, 0u);
        bits4[2 * l + 1] = make_uint4(0u, 0u, 0u, 0u);
        if (l < G::NW / 32) S.dupw[l] = 0u;
#pragma unroll
        for (int q = 0; q < (NC * WAVE + 511) / 512; ++q)
            reinterpret_cast<uint64_t*>(S.mk)[q * WAVE + l] = ~0ull;
        wsync();
        if (cnt > 0) S.mk[off] = (int8_t)l;
        wsync();
        // lane -> A entry of each product (marker bytes + DPP max scans carried across chunks)
        int src[NC];
        {
            int mrk[NC];
#pragma unroll
            for (int r = 0; r < NC; ++r) mrk[r] = S.mk[r * WAVE + l];
            int carry = -1;
#pragma unroll
            for (int r = 0; r < NC; ++r) {
                src[r] = max(wave_incl_max_dpp(mrk[r]), carry);
                carry = readlane_i(src[r], WAVE - 1);
            }
        }
        IP idx[NC];
#pragma unroll
        for (int r = 0; r < NC; ++r) {
            const int t = r * WAVE + l;
            idx[r] = t < P ? S.jb0[src[r]] + (IP)(t - S.joff[src[r]]) : (IP)0;
        }
        // every product of the row in flight at once (int32 row pointers: 32-bit byte
        // offsets from a scalar base -- the host keeps B under 2^29 entries on this path)
        int col[NC];
#pragma unroll
        for (int r = 0; r < NC; ++r) col[r] = ld_idx(Bj, idx[r]);
        T prd[NC];
        if (VALS) {
            T bx[NC];
#pragma unroll
            for (int r = 0; r < NC; ++r) bx[r] = ld_idx(Bx, idx[r]);
#pragma unroll
            for (int r = 0; r < NC; ++r) prd[r] = mul_rn(S.ja[src[r]], bx[r]);
        }
#pragma unroll
        for (int r = 0; r < NC; ++r)
            if (r * WAVE + l >= P) col[r] = -1;
        // column bits; a product whose bit was already set flags its word
        uint32_t dupb = 0;
#pragma unroll
        for (int r = 0; r < NC; ++r) {
            const int cc = col[r] < 0 ? 0 : col[r];
            const uint32_t bit = col[r] < 0 ? 0u : 1u << (cc & 31);
            if (atomicOr(&S.bits[cc >> 5], bit) & bit) dupb |= 1u << r;
        }
        const bool anydup = __ballot(dupb != 0u) != 0ull;
        if (anydup) {
#pragma unroll
            for (int r = 0; r < NC; ++r)
                if ((dupb >> r) & 1u) atomicOr(&S.dupw[col[r] >> 10], 1u << ((col[r] >> 5) & 31));
        }
        wsync();
        // popcount prefix over this lane's 8 contiguous words, word flags in bit 15
        int nnz;
        {
            const uint4 q0 = bits4[2 * l], q1 = bits4[2 * l + 1];
            const int c0 = __popc(q0.x), c1 = __popc(q0.y), c2 = __popc(q0.z), c3 = __popc(q0.w);
            const int c4 = __popc(q1.x), c5 = __popc(q1.y), c6 = __popc(q1.z), c7 = __popc(q1.w);
            const int mine = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
            const int pincl = wave_incl_sum_dpp(mine);
            nnz = readlane_i(pincl, WAVE - 1);
            const uint32_t fl = anydup ? (S.dupw[l >> 2] >> ((l & 3) * 8)) & 0xffu : 0u;
            const int p0 = pincl - mine, p1 = p0 + c0, p2 = p1 + c1, p3 = p2 + c2, p4 = p3 + c3,
                      p5 = p4 + c4, p6 = p5 + c5, p7 = p6 + c6;
            auto f = [&](int p, int i) { return (uint32_t)p | (((fl >> i) & 1u) << 15); };
            uint4 w;
            w.x = f(p0, 0) | (f(p1, 1) << 16);
            w.y = f(p2, 2) | (f(p3, 3) << 16);
            w.z = f(p4, 4) | (f(p5, 5) << 16);
            w.w = f(p6, 6) | (f(p7, 7) << 16);
            reinterpret_cast<uint4*>(S.wpre)[l] = w;
        }
        wsync();
        // products in flagged words: their number decides the spill; (VALS) their list
        int L = 0;
        int pos[NC];   // output position, | 1 << 30 in a flagged word; -1: no product
        if (VALS) {
#pragma unroll
            for (int r = 0; r < NC; ++r) {
                const int cc = col[r] < 0 ? 0 : col[r];
                const uint32_t pw = S.wpre[cc >> 5];
                const int p = (int)(pw & 0x7fffu) + __popc(S.bits[cc >> 5] & ((1u << (cc & 31)) - 1u));
                pos[r] = col[r] < 0 ? -1 : (p | (int)((pw >> 15) << 30));
            }
            if (anydup) {
#pragma unroll
                for (int r = 0; r < NC; ++r) {
                    const bool fg = pos[r] >= 0 && (pos[r] >> 30);
                    const unsigned long long m = __ballot(fg);
                    if (m) {
                        const int slot = L + lane_rank(m);
                        if (fg && slot < G::LCAP) {
                            S.lp[slot] = pos[r] & 0x3fffffff;
                            S.lc[slot] = col[r];
                            S.lx[slot] = prd[r];
                        }
                        L += (int)__popcll(m);
                    }
                }
            }
        } else if (anydup) {
#pragma unroll
            for (int r = 0; r < NC; ++r) {
                const bool fg = col[r] >= 0 && ((S.dupw[col[r] >> 10] >> ((col[r] >> 5) & 31)) & 1u);
                L += (int)__popcll(__ballot(fg));
            }
        }
        const bool take = L <= G::LCAP;
        if (MODE == ROW_SYM) {
            if (take) {
                if (l == 0) row_cnt[row] = nnz;
            } else {
                spill_row();
            }
            return;
        }
        if (LB) lb_publish(nnz);
        if (!take) {
            spill_row();
            if (LB) lb_base(nnz);
            return;
        }
        // the first list entry of each position sums its position's entries in list order
        bool lead = false;
        int lpos = 0, lcol = 0;
        T lsum = (T)0;
        if (L > 0) {
            wsync();
            T x = (T)0;
            if (l < L) {
                lpos = S.lp[l];
                lcol = S.lc[l];
                x = S.lx[l];
            }
            lead = l < L;
            for (int j = 0; j < L; ++j) {
                const int pj = __builtin_amdgcn_readlane(lpos, j);
                const T xj = readlane_v(x, j);
                if (pj == lpos) {
                    if (j < l) lead = false;
                    else lsum = add_rn(lsum, xj);
                }
            }
        }
        const int64_t base = LB ? lb_base(nnz) : (int64_t)Coff[row];
        if (base < 0) return;
        int32_t* __restrict__ crow = Cj + base;
        T* __restrict__ xrow = Cx + base;
#pragma unroll
        for (int r = 0; r < NC; ++r) {
            if (pos[r] >= 0 && !(pos[r] >> 30)) {
                crow[pos[r]] = col[r];
                xrow[pos[r]] = scale(alpha, add_rn((T)0, prd[r]));
            }
        }
        if (lead) {
            crow[lpos] = lcol;
            xrow[lpos] = scale(alpha, lsum);
        }
    };

    if (fits && P > 0) {
        switch (((P + WAVE - 1) / WAVE + 1) >> 1) {
            case 1: row_body(IntC<2>{}); break;
            case 2: row_body(IntC<4>{}); break;
            case 3: row_body(IntC<6>{}); break;
            case 4: row_body(IntC<8>{}); break;
            default: row_body(IntC<10>{}); break;
        }
        return;
    }
    static_assert(G::R == 10, "row_body dispatch covers 10 chunks");

    // ---- empty rows, and rows for the general kernel (> 64 A entries or > PREG products)
    const bool empty = nA <= 0 || ncols <= 0 || (fits && P == 0);
    if (MODE == ROW_SYM) {
        if (empty) {
            if (l == 0) row_cnt[row] = 0;
        } else {
            spill_row();
        }
        return;
    }
    if (!LB) {
        if (!empty) spill_row();
        return;
    }
    // LB: a spilled row still needs its count -- 64 A entries at a time, chunk by chunk
    int64_t nnz = 0;
    if (!empty) {
        bits4[2 * l] = make_uint4(0u, 0u, 0u, 0u);
        bits4[2 * l + 1] = make_uint4(0u, 0u, 0u, 0u);
        wsync();
        for (int b = 0; b < nA; b += WAVE) {
            int bc = 0;
            IP bb = 0;
            if (b + l < nA) {
                const int32_t k = Aj[a0 + b + l];
                bb = Bp[k];
                bc = (int)(Bp[k + 1] - bb);
            }
            const int bincl = wave_incl_sum(bc);
            const int boff = bincl - bc;
            const int bP = readlane_i(bincl, WAVE - 1);
            S.jb0[l] = bb;
            S.joff[l] = boff;
            int carry = -1;
            for (int c0 = 0; c0 < bP; c0 += WAVE) {
                S.marker[l] = -1;
                wsync();
                if (bc > 0 && boff >= c0 && boff < c0 + WAVE) S.marker[boff - c0] = (int8_t)l;
                wsync();
                const int src = max(wave_incl_max_dpp((int)S.marker[l]), carry);
                carry = readlane_i(src, WAVE - 1);
                const int t = c0 + l;
                if (t < bP) set_bit(S.bits, Bj[S.jb0[src] + (IP)(t - S.joff[src])]);
            }
            wsync();
        }
        const uint4 q0 = bits4[2 * l], q1 = bits4[2 * l + 1];
        const int mine = __popc(q0.x) + __popc(q0.y) + __popc(q0.z) + __popc(q0.w) + __popc(q1.x) +
                         __popc(q1.y) + __popc(q1.z) + __popc(q1.w);
        nnz = wave_sum64(mine);
        spill_row();
    }
    lb_publish(nnz);
    lb_base(nnz);
}

}  // namespace spg
