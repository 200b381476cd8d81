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
//           is final (0 + a*b, scipy's sum starts at 0) and goes from registers to its
//           position in an LDS stage, which leaves for C in position order (coalesced).
//           Products in flagged words (typically ~3 % of them) are compacted, in product
//           order, into a list of <= LCAP entries; lane i of the list sums, in list order,
//           every entry of its position if it is the first one (readlane loop, no atomics),
//           and stages that column.
//
// So no product waits on another product: the LDS owner rounds of k_short (which order
// every accumulate) are gone from the common case.  Rows the kernel cannot take (> 64 A
// entries, > PREG products, > LCAP products in flagged words) are spilled -- by the same
// predicate in every mode, so the symbolic and numeric passes spill the same rows -- to the
// general kernel (k_symbolic / k_numeric over the spill list).
//
// MODES: ROW_SYM counts (ALG2/3 symbolic, and ALG1's count pass, which also leaves every
// A entry's B row extent behind for the numeric pass), ROW_NUM writes at C's row pointer
// (ALG2/3 numeric), ROW_LB is ALG1's numeric pass with the row-pointer scan inside it: its
// first blocks scan the count pass's row counts (C's row pointer, one published prefix per
// 64-row group, the host mirror), the rest take the rows, each at its group's prefix plus
// the counts before it in the group (RowScan).  Spilled rows are counted by the count pass
// (the count-only loop below) and get their values from a k_numeric launch over the spill
// list afterwards.
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
    static constexpr int MKC = 16;                    // marker bytes per lane (>= R)
    static constexpr int MKB = WAVE * MKC;            // marker bytes
    static_assert(LCAP <= WAVE, "one list entry per lane");
};
using RowSmall = RowCfg<10, 64, 4>;

// One record per A entry, read with one wide LDS access per chunk (16 B for int32 row
// pointers and f64 values).
template <typename T, typename IP, bool VALS> struct alignas(VALS ? (sizeof(IP) + 4 + sizeof(T) >= 16 ? 16 : 8) : 8) JRec {
    IP jb0;         // B row start
    int32_t joff;   // first flattened product
    T ja;           // A value (VALS)
};
template <typename T, typename IP> struct alignas(8) JRec<T, IP, false> {
    IP jb0;
    int32_t joff;
};

template <typename T, typename IP, typename G, bool VALS, int SCAP = 0> struct RowLds {
    union {                        // the bitmap, expanded in place after pass 1 into
        uint32_t bits[G::NW];      //   (word, exclusive popcount prefix | 0x8000 for a
        uint2 bw[VALS ? G::NW : 1];   // flagged word): one 8-byte read gives a position
    };                             //   (numeric only: counting needs the bitmap alone)
    uint32_t dupw[G::NW / 32];     // one bit per bitmap word: a column of it was hit twice
    JRec<T, IP, VALS> jr[WAVE];    // per A entry: B row start, first product, value
    union {                        // phases of one row that never overlap:
        uint8_t mk[G::MKB];        //   lane -> A-entry markers of every chunk (pass 1),
                                   //   transposed: product t at 16 * (t % 64) + t / 64
        struct {                   //   flagged-word products in product order (fix-up)
            T lx[VALS ? G::LCAP : 1];
            int32_t lc[VALS ? G::LCAP : 1];
            int32_t lp[VALS ? G::LCAP : 1];
        };
        int8_t marker[WAVE + 4];   //   count-only loop (one chunk at a time)
    };
    // ALG1 numeric with the scan inside: the row's group word and in-group count prefix,
    // parked here (not in registers) until the row's output is ready
    unsigned long long lb_gw;
    long long lb_gsum;
};

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

// One row's result, held in registers until its base is known.  cp[r] packs the column
// (bits 0..13), the output position (bits 14..27) and the flagged-word bit (28) of this
// lane's product of chunk r; -1: no product.  List leaders (lcol >= 0) own the column lcol
// at position lpos with the sum lsum.
constexpr int CP_POS = 14;
constexpr int CP_FLAG = 1 << 28;
template <typename T, int NCMAX> struct RowOut {
    int cp[NCMAX];
    T prd[NCMAX];
    T lsum;
    int lpos, lcol;
    int nnz;
    bool take;
};

// A row's front: lane l loads its A entry, its value and its B row extent (registers only,
// so the next row's front can be in flight while the current row is worked on).
template <typename T, typename IP> struct RowFront {
    IP b0;
    int cnt;
    T av;
};
template <bool VALS, typename T, typename IP>
__device__ __forceinline__ RowFront<T, IP> row_front_load(int l, int64_t a0, int nA, const int32_t* __restrict__ Aj,
                                                          const T* __restrict__ Ax, const IP* __restrict__ Bp) {
    RowFront<T, IP> f{(IP)0, 0, (T)0};
    if (l < nA) {
        const int32_t k = Aj[a0 + l];
        f.b0 = Bp[k];
        f.cnt = (int)(Bp[k + 1] - f.b0);
        if (VALS) f.av = Ax[a0 + l];
    }
    return f;
}
// ALG1: the count pass leaves every A entry's B row extent behind (RowExt, parallel to A's
// entries), so the numeric pass reads it in one load instead of A's column and then B's
// row pointer (one dependent global load less per row).
template <typename IP> struct alignas(sizeof(IP) == 8 ? 16 : 8) RowExt {
    IP b0;
    int32_t cnt;
};
template <bool VALS, typename T, typename IP>
__device__ __forceinline__ RowFront<T, IP> row_front_ext(int l, int64_t a0, int nA, const RowExt<IP>* __restrict__ ext,
                                                         const T* __restrict__ Ax) {
    RowFront<T, IP> f{(IP)0, 0, (T)0};
    if (l < nA) {
        const RowExt<IP> e = ext[a0 + l];
        f.b0 = e.b0;
        f.cnt = e.cnt;
        if (VALS) f.av = Ax[a0 + l];
    }
    return f;
}

// ALG1 numeric pass with the row-pointer scan inside it: blocks 0..nscan-1 scan the count
// pass's row counts (scan_tile: C's row pointer, the total, the host mirror) and publish the
// exclusive prefix of every 64-row group in gpre; the other blocks take the rows, each
// row's offset = its group's prefix + the counts of the rows before it in the group.  A row
// wave reads its group word when it starts and waits for it only when its output is ready
// to leave (by then the scan is long done: it reads 8 bytes per row).  The scan blocks come
// first in dispatch order and wait on nothing the row blocks produce.
template <typename OFF> struct RowScan {
    int64_t nscan;                     // scan tiles; 0: offsets come from Coff
    OFF* out;                          // C's row pointer
    unsigned long long* status;        // ticket word + tile status words, zero on entry
    unsigned long long* gpre;          // group prefixes, zero on entry
    int64_t* scalars;
    int32_t* move_cnt;
    int64_t* move_dst;
    int64_t* host_mirror;
    int64_t mirror_gen;
    int mirror_n;
    uint64_t spin;                     // bound of every wait, wall-clock ticks (SCAN_SPIN)
};

// the exclusive prefix of a row group: its published word.  The scan tiles take tickets in
// the order they start and wait on nothing the row blocks produce, so the word arrives; a
// wait past `spin` ticks (a scan tile not scheduled, which no dispatch order should cause)
// stops and sums the group's preceding row counts directly -- same value, and the wave
// always finishes.  The wait stays in scalar registers (the row's output occupies the vector
// registers).
__device__ __forceinline__ long long row_group_prefix(const unsigned long long* gp, unsigned long long gw,
                                                      const int64_t* cnt, int64_t g0, uint64_t spin) {
    if (spin == 0) return wave_direct_sum(cnt, g0);   // (the direct path, for the tests)
    uint64_t t0 = 0;   // (the clock is read only once the word is found not ready)
    while (!(gw & GPRE_READY)) {
        const uint64_t now = wall_clock64();
        if (t0 == 0) t0 = now;
        else if (now - t0 > spin) return wave_direct_sum(cnt, g0);
        __builtin_amdgcn_s_sleep(2);
        const unsigned long long v = __hip_atomic_load(gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        gw = ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
             (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    }
    return (long long)(gw & SCAN_VMASK);
}

// ... then the flattened product offset of each entry goes to LDS.  Returns the row's
// product count P (wave-uniform).
template <bool VALS, typename T, typename IP, typename Lds>
__device__ __forceinline__ int row_front_commit(Lds& S, int l, const RowFront<T, IP>& f, int& off) {
    const int incl = wave_incl_sum_dpp(f.cnt);
    off = incl - f.cnt;
    if constexpr (VALS) S.jr[l] = JRec<T, IP, VALS>{f.b0, off, f.av};
    else S.jr[l] = JRec<T, IP, VALS>{f.b0, off};
    return readlane_i(incl, WAVE - 1);
}

// The register path for a row of P (1 <= P <= NC*64) products: bitmap, positions, the
// flagged-word list and its fix-up.  o.take = false when the list overflows LCAP (the row
// then goes to the general kernel; o.nnz is still its count).
template <int NC, bool VALS, bool AVL, typename T, typename IP, typename G, typename Lds, int NCMAX>
__device__ __forceinline__ void row_pass(Lds& S, int l, int cnt, int off, int P, const int32_t* __restrict__ Bj,
                                         const T* __restrict__ Bx, RowOut<T, NCMAX>& o) {
    static_assert(NC <= NCMAX, "chunks");
    uint4* bits4 = reinterpret_cast<uint4*>(S.bits);
    bits4[2 * l] = make_uint4(0u, 0u, 0u, 0u);
    bits4[2 * l + 1] = make_uint4(0u, 0u, 0u, 0u);
    if (l < G::NW / 32) S.dupw[l] = 0u;
    static_assert(NC <= G::MKC, "one marker byte per chunk and lane");
    reinterpret_cast<uint4*>(S.mk)[l] = make_uint4(0u, 0u, 0u, 0u);
    wsync();
    if (cnt > 0) S.mk[((off & (WAVE - 1)) * G::MKC) | (off >> 6)] = (uint8_t)(l + 1);
    wsync();
    // lane -> A entry + 1 of each product (marker bytes + DPP max scans carried across
    // chunks; the first product always has a marker, so every src >= 1); a lane's markers
    // of all chunks come with one 16-byte LDS read
    unsigned src[NC];
    {
        const uint4 m4 = reinterpret_cast<const uint4*>(S.mk)[l];
        const uint32_t mw[4] = {m4.x, m4.y, m4.z, m4.w};
        unsigned mrk[NC];
#pragma unroll
        for (int r = 0; r < NC; ++r) mrk[r] = (mw[r >> 2] >> (8 * (r & 3))) & 0xffu;
        unsigned carry = 0;
#pragma unroll
        for (int r = 0; r < NC; ++r) {
            src[r] = max(wave_incl_umax_dpp(mrk[r]), carry);
            carry = (unsigned)readlane_i((int)src[r], WAVE - 1);
        }
    }
    const JRec<T, IP, VALS>* jr1 = S.jr - 1;   // indexed by src
    IP idx[NC];
    T av[NC];
#pragma unroll
    for (int r = 0; r < NC; ++r) {
        const int t = r * WAVE + l;
        JRec<T, IP, VALS> j;
        if constexpr (sizeof(j) == 16) {   // one ds_read_b128
            const uint4 q = *reinterpret_cast<const uint4*>(&jr1[src[r]]);
            __builtin_memcpy(&j, &q, 16);
        } else {
            j = jr1[src[r]];
        }
        idx[r] = t < P ? j.jb0 + (IP)(t - j.joff) : (IP)0;
        if constexpr (VALS && !AVL) av[r] = j.ja;
    }
    // every product of the row in flight at once
    int col[NC];
#pragma unroll
    for (int r = 0; r < NC; ++r) col[r] = ld_idx(Bj, idx[r]);
    if constexpr (VALS) {
        T bx[NC];
#pragma unroll
        for (int r = 0; r < NC; ++r) bx[r] = ld_idx(Bx, idx[r]);
        // (AVL) A's values from LDS while the gathers are in flight, not held in registers
        // across them
#pragma unroll
        for (int r = 0; r < NC; ++r) {
            if constexpr (AVL) o.prd[r] = mul_rn(jr1[src[r]].ja, bx[r]);
            else o.prd[r] = mul_rn(av[r], bx[r]);
        }
    }
#pragma unroll
    for (int r = 0; r < NC; ++r)
        if (r * WAVE + l >= P) col[r] = -1;
    // column bits; a product whose bit was already set flags its word
    uint32_t dupb = 0;
    int ndup = 0;   // products whose column was already set (wave total)
#pragma unroll
    for (int r = 0; r < NC; ++r) {
        const int cc = col[r] < 0 ? 0 : col[r];
        const uint32_t bit = col[r] < 0 ? 0u : 1u << (cc & 31);
        const bool hit = (atomicOr(&S.bits[cc >> 5], bit) & bit) != 0u;
        if (hit) dupb |= 1u << r;
        if (!VALS) ndup += (int)__popcll(__ballot(hit));
    }
    const bool anydup = VALS ? __ballot(dupb != 0u) != 0ull : ndup > 0;
    if (anydup) {
#pragma unroll
        for (int r = 0; r < NC; ++r)
            if ((dupb >> r) & 1u) atomicOr(&S.dupw[col[r] >> 10], 1u << ((col[r] >> 5) & 31));
    }
    wsync();
    // (counting) distinct columns = products - repeated hits: no bitmap popcount
    if (!VALS) o.nnz = P - ndup;
    // popcount prefix over this lane's 8 contiguous words, word flags in bit 15; the words
    // and their prefixes go back as (word, prefix) pairs over the same LDS (every lane's
    // reads are one instruction ahead of any lane's writes)
    if constexpr (VALS) {
        const uint4 q0 = bits4[2 * l], q1 = bits4[2 * l + 1];
        const int c0 = __popc(q0.x), c1 = __popc(q0.y), c2 = __popc(q0.z), c3 = __popc(q0.w);
        const int c4 = __popc(q1.x), c5 = __popc(q1.y), c6 = __popc(q1.z), c7 = __popc(q1.w);
        const int mine = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
        const int pincl = wave_incl_sum_dpp(mine);
        o.nnz = readlane_i(pincl, WAVE - 1);
        const uint32_t fl = anydup ? (S.dupw[l >> 2] >> ((l & 3) * 8)) & 0xffu : 0u;
        const int p0 = pincl - mine, p1 = p0 + c0, p2 = p1 + c1, p3 = p2 + c2, p4 = p3 + c3,
                  p5 = p4 + c4, p6 = p5 + c5, p7 = p6 + c6;
        auto f = [&](int p, int i) { return (uint32_t)p | (((fl >> i) & 1u) << 15); };
        wsync();
        uint4* bw4 = reinterpret_cast<uint4*>(S.bw);
        bw4[4 * l + 0] = make_uint4(q0.x, f(p0, 0), q0.y, f(p1, 1));
        bw4[4 * l + 1] = make_uint4(q0.z, f(p2, 2), q0.w, f(p3, 3));
        bw4[4 * l + 2] = make_uint4(q1.x, f(p4, 4), q1.y, f(p5, 5));
        bw4[4 * l + 3] = make_uint4(q1.z, f(p6, 6), q1.w, f(p7, 7));
        wsync();
    }
    // products in flagged words: their number decides the spill; (VALS) their list
    int L = 0;
#pragma unroll
    for (int r = NC; r < NCMAX; ++r) o.cp[r] = -1;
    if (VALS) {
#pragma unroll
        for (int r = 0; r < NC; ++r) {
            const int cc = col[r] < 0 ? 0 : col[r];
            const uint2 bw = S.bw[cc >> 5];
            const int p = (int)(bw.y & 0x7fffu) + __popc(bw.x & ((1u << (cc & 31)) - 1u));
            o.cp[r] = col[r] < 0 ? -1 : (cc | (p << CP_POS) | (int)(((bw.y >> 15) & 1u) << 28));
        }
        if (anydup) {
#pragma unroll
            for (int r = 0; r < NC; ++r) {
                const bool fg = o.cp[r] >= 0 && (o.cp[r] & CP_FLAG);
                const unsigned long long m = __ballot(fg);
                if (m) {
                    const int slot = L + lane_rank(m);
                    if (fg && slot < G::LCAP) {
                        S.lp[slot] = (o.cp[r] >> CP_POS) & 0x3fff;
                        S.lc[slot] = o.cp[r] & 0x3fff;
                        S.lx[slot] = o.prd[r];
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
    o.take = L <= G::LCAP;
    // the first list entry of each position sums its position's entries in list order
    o.lcol = -1;
    o.lpos = 0;
    o.lsum = (T)0;
    if (VALS && o.take && L > 0) {
        wsync();
        T x = (T)0;
        int lp = -1, lc = -1;
        if (l < L) {
            lp = S.lp[l];
            lc = S.lc[l];
            x = S.lx[l];
        }
        bool lead = l < L;
        T sum = (T)0;
        for (int j = 0; j < L; ++j) {
            const int pj = __builtin_amdgcn_readlane(lp, j);
            const T xj = readlane_v(x, j);
            if (pj == lp) {
                if (j < l) lead = false;
                else sum = add_rn(sum, xj);
            }
        }
        o.lcol = lead ? lc : -1;
        o.lpos = lp;
        o.lsum = sum;
    }
}

// P in [1, PREG]: the register path with the smallest chunk count that holds P, then
// `then(o)` on its result -- inside each case, so the result of one case
// never meets another's at a join (it would otherwise occupy registers for all five).
template <bool VALS, bool AVL, typename T, typename IP, typename G, typename Lds, typename F>
__device__ __forceinline__ void row_dispatch(Lds& S, int l, int cnt, int off, int P, const int32_t* __restrict__ Bj,
                                             const T* __restrict__ Bx, F&& then) {
    static_assert(G::R == 10, "dispatch covers 10 chunks");
    auto run = [&](auto nct) {
        constexpr int NC = decltype(nct)::value;
        RowOut<T, NC> o;
        row_pass<NC, VALS, AVL, T, IP, G>(S, l, cnt, off, P, Bj, Bx, o);
        then(o);
    };
    switch ((P + WAVE - 1) / WAVE) {   // exact chunk counts where rows are common
        case 1:
        case 2: run(IntC<2>{}); break;
        case 3: run(IntC<3>{}); break;
        case 4: run(IntC<4>{}); break;
        case 5: run(IntC<5>{}); break;
        case 6: run(IntC<6>{}); break;
        case 7: run(IntC<7>{}); break;
        case 8: run(IntC<8>{}); break;
        default: run(IntC<10>{}); break;
    }
}

// The row's outputs (unflagged products, then the list leaders) through LDS: every entry goes
// to its position in a stage built over the wave's (now free) bitmap / prefix / record area,
// then the row leaves in position order, 64 consecutive entries per store instead of 64
// scattered ones (scattered 4/8-byte stores cost the L1 one tag lookup per line touched:
// measured 6.6 us of the 33 us numeric pass on config 2, 1.8 us saved).  Rows longer than
// the stage take several windows.
template <bool UNIT, typename T, int NCMAX, typename Lds>
__device__ __forceinline__ void row_write_staged(Lds& S, int l, const RowOut<T, NCMAX>& o,
                                                 int32_t* __restrict__ crow, T* __restrict__ xrow, T alpha) {
    constexpr int W = (int)(__builtin_offsetof(Lds, lb_gw) / (sizeof(T) + 4));
    T* sv = reinterpret_cast<T*>(&S);
    int32_t* sc = reinterpret_cast<int32_t*>(sv + W);
    wsync();   // row_pass's reads of these words are done
    for (int w0 = 0; w0 < o.nnz; w0 += W) {
#pragma unroll
        for (int r = 0; r < NCMAX; ++r) {
            const int c = o.cp[r];
            const int p = ((c >> CP_POS) & 0x3fff) - w0;
            if (c >= 0 && !(c & CP_FLAG) && (unsigned)p < (unsigned)W) {
                sc[p] = c & 0x3fff;
                const T v = add_rn((T)0, o.prd[r]);
                sv[p] = UNIT ? v : mul_rn(alpha, v);
            }
        }
        if (o.lcol >= 0 && (unsigned)(o.lpos - w0) < (unsigned)W) {
            sc[o.lpos - w0] = o.lcol;
            sv[o.lpos - w0] = UNIT ? o.lsum : mul_rn(alpha, o.lsum);
        }
        wsync();
        const int n = min(W, o.nnz - w0);
        for (int i = l; i < n; i += WAVE) {
            crow[w0 + i] = sc[i];
            xrow[w0 + i] = sv[i];
        }
        wsync();
    }
}
template <typename T, int NCMAX, typename Lds>
__device__ __forceinline__ void row_write(Lds& S, int l, const RowOut<T, NCMAX>& o, int32_t* __restrict__ crow,
                                          T* __restrict__ xrow, T alpha) {
    if (alpha == (T)1) row_write_staged<true>(S, l, o, crow, xrow, alpha);   // (uniform branch)
    else row_write_staged<false>(S, l, o, crow, xrow, alpha);
}

// Structural nnz of any row with <= 16384 columns: 64 A entries at a time, chunk by chunk
// (ALG1 single pass: the count of a row the register path cannot take).
template <typename IP, typename Lds>
__device__ int row_count_only(Lds& S, int l, int64_t a0, int nA, const int32_t* __restrict__ Aj,
                              const IP* __restrict__ Bp, const int32_t* __restrict__ Bj) {
    uint4* bits4 = reinterpret_cast<uint4*>(S.bits);
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
        S.jr[l].jb0 = bb;
        S.jr[l].joff = boff;
        int carry = -1;
        for (int c0 = 0; c0 < bP; c0 += WAVE) {
            S.marker[l] = -1;
            wsync();
            if (bc > 0 && boff >= c0 && boff < c0 + WAVE) S.marker[boff - c0] = (int8_t)l;
            wsync();
            const int src = max(wave_incl_max_dpp((int)S.marker[l]), carry);
            carry = readlane_i(src, WAVE - 1);
            const int t = c0 + l;
            if (t < bP) set_bit(S.bits, Bj[S.jr[src].jb0 + (IP)(t - S.jr[src].joff)]);
        }
        wsync();
    }
    const uint4 q0 = bits4[2 * l], q1 = bits4[2 * l + 1];
    const int mine = __popc(q0.x) + __popc(q0.y) + __popc(q0.z) + __popc(q0.w) + __popc(q1.x) + __popc(q1.y) +
                     __popc(q1.z) + __popc(q1.w);
    return (int)wave_sum64(mine);
}

// ---- one wave per row.
//   ROW_SYM (ALG2/3 symbolic): the row's count into row_cnt, or the row to the spill list
//     (the general kernel counts it).  With ROW_COUNT_ALL (ALG1 count pass) every row's
//     count goes to row_cnt -- a row the register path cannot take is counted by
//     row_count_only -- and the spill list holds the rows whose VALUES the general kernel
//     computes.
//   ROW_NUM: values at C's row pointer Coff (none when scan_scal[1] says the scan of an
//     int32 row pointer overflowed).  Spilled rows are appended to the spill list
//     (the same predicate spilled them in the symbolic pass) unless ROW_LISTED (ALG1: the
//     count pass listed them).  cap > 0 (ALG1, C's arrays hold `cap` entries): a row that
//     would end past cap writes nothing (the host sees the total and redoes the product).
enum { ROW_COUNT_ALL = 1, ROW_LISTED = 2 };
#ifndef SPG_ROW_PAIR
#define SPG_ROW_PAIR 1
#endif
#ifndef SPG_ROW_PAIR_SYM
#define SPG_ROW_PAIR_SYM 1
#endif
// rows per wave, per mode.  Two rows per wave in the count pass (42 VGPRs, still 8 waves per
// SIMD: config 2's 16384 rows become one generation of 8192 resident waves) measured no
// gain (12.7 vs 12.1 us; three rows 15 us): the count pass is bound by its ~370 VALU
// instructions per row, not by the dependent-load chain
template <int MODE> constexpr int row_pair() { return MODE == 0 ? SPG_ROW_PAIR_SYM : SPG_ROW_PAIR; }
// A's values re-read from LDS after the gathers instead of held in registers across them
// (ROW_LB only): fewer live registers, but measured 1.5 us slower on config 2's numeric pass
#ifndef SPG_ROW_AVLDS
#define SPG_ROW_AVLDS 0
#endif
// register budget: 5 waves per SIMD (<= 96 VGPRs) for 4- and 8-byte values
template <typename T, typename IP, typename OFF, int MODE, typename G>
__global__ __launch_bounds__(G::WPB * WAVE, sizeof(T) <= 8 ? 5 : 3) void k_row(
    int64_t row0, int64_t nrows, int64_t ncols, const IP* __restrict__ Ap,
    const int32_t* __restrict__ Aj, const T* __restrict__ Ax, const IP* __restrict__ Bp,
    const int32_t* __restrict__ Bj, const T* __restrict__ Bx, const OFF* __restrict__ Coff,
    int32_t* __restrict__ Cj, T* __restrict__ Cx, T alpha, int64_t* __restrict__ row_cnt,
    int32_t* __restrict__ spill, int32_t* __restrict__ spill_count, int flags, int64_t cap,
    const int64_t* __restrict__ scan_scal, unsigned long long* __restrict__ zero_words, int64_t nzero,
    RowExt<IP>* __restrict__ ext, RowScan<OFF> sa) {
    static_assert(MODE == ROW_SYM || MODE == ROW_NUM || MODE == ROW_LB, "modes");
    static_assert(G::WPB * WAVE == BLOCK, "scan tiles are blocks of BLOCK threads");
    constexpr bool VALS = MODE != ROW_SYM;
    constexpr bool lb = MODE == ROW_LB;
    constexpr bool AVL = lb && SPG_ROW_AVLDS;
    constexpr int RP = row_pair<MODE>();
    __shared__ __attribute__((aligned(16))) RowLds<T, IP, G, VALS> lds[G::WPB];
    // (ALG1 count pass) the next launch's scan status words are zeroed here: no memset
    if (zero_words)
        for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < nzero; i += (int64_t)gridDim.x * BLOCK)
            zero_words[i] = 0ull;
    if (lb && (int64_t)blockIdx.x < sa.nscan) {
        // a scan block scans the tile of the ticket it takes (tickets follow the order the
        // scan blocks start, so every tile's predecessors have started: the look-back ends)
        __shared__ ScanLds scan_l;
        __shared__ int64_t ticket;
        if (threadIdx.x == 0) ticket = (int64_t)atomicAdd(&sa.status[0], 1ull);
        __syncthreads();
        scan_tile<OFF, int64_t>(ticket, nrows, row_cnt + row0, sa.out, sa.status + 1, sa.scalars,
                                sa.move_cnt, sa.move_dst, sa.host_mirror, sa.mirror_gen, sa.mirror_n,
                                nullptr, scan_l, sa.gpre, sa.spin);
        return;
    }
    const int l = lane_id();
    const int wv = uniform((int)(threadIdx.x >> 6));
    RowLds<T, IP, G, VALS>& S = lds[wv];
    const bool count_all = MODE == ROW_SYM && (flags & ROW_COUNT_ALL);
    // ROW_PAIR consecutive rows per wave: both rows' fronts (A entries, B row extents) are
    // loaded before the first row is worked on, so the second row's dependent loads are
    // in flight during the first row's gathers and LDS work
    const int64_t it0 = (((int64_t)blockIdx.x - (lb ? sa.nscan : 0)) * G::WPB + wv) * RP;
    if (it0 >= nrows) return;
    const int nr = (int)min((int64_t)RP, nrows - it0);
    int64_t a0s[RP + 1];
#pragma unroll
    for (int q = 0; q <= RP; ++q) a0s[q] = q <= nr ? (int64_t)Ap[row0 + it0 + q] : 0;
    RowFront<T, IP> fr[RP];
#pragma unroll
    for (int q = 0; q < RP; ++q) {
        const int nAq = q < nr ? (int)(a0s[q + 1] - a0s[q]) : 0;
        const bool f = nAq > 0 && nAq <= WAVE && ncols > 0;
        if (lb) {
            fr[q] = row_front_ext<VALS, T, IP>(l, a0s[q], f ? nAq : 0, ext, Ax);
        } else {
            fr[q] = row_front_load<VALS, T, IP>(l, a0s[q], f ? nAq : 0, Aj, Ax, Bp);
            if (MODE == ROW_SYM && ext && f && l < nAq) ext[a0s[q] + l] = RowExt<IP>{fr[q].b0, fr[q].cnt};
        }
    }
    // (lb) each row's group word and the counts of the rows before it in its group
    unsigned long long gw[RP] = {};
    int gc[RP] = {};   // (a row's count < 2^31: the low word of its int64 count)
    if (lb) {
#pragma unroll
        for (int q = 0; q < RP; ++q) {
            gw[q] = 0;
            gc[q] = 0;
            if (q < nr) {
                const int64_t it = it0 + q, g0 = it & ~(int64_t)(WAVE - 1);
                gw[q] = __hip_atomic_load(&sa.gpre[it >> 6], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                gc[q] = g0 + l < it ? reinterpret_cast<const int*>(row_cnt + row0 + g0 + l)[0] : 0;
            }
        }
    }

    auto do_row = [&](int64_t row, int64_t a0, int nA, const RowFront<T, IP>& f, unsigned long long gwq,
                      int gcq) {
        int64_t base = 0;
        bool room = true;
        // (lb) wave-uniform from here on (scalar registers): the group word and the counts
        // of the rows before this one in its group
        if (lb) {
            const int gsum = wave_incl_sum_dpp(gcq);
            if (l == WAVE - 1) {
                S.lb_gw = gwq;
                S.lb_gsum = gsum;
            }
        }
        if (MODE == ROW_NUM) {
            base = (int64_t)Coff[row];
            if (cap > 0) room = (int64_t)Coff[row + 1] <= cap;
            // (ALG1) an int32 row pointer that overflowed (scan scalars[1]) is not an offset
            if (scan_scal && scan_scal[1]) room = false;
        }
        int off = 0, P = 0;
        bool fits = nA > 0 && nA <= WAVE && ncols > 0;
        if (fits) {
            P = row_front_commit<VALS, T, IP>(S, l, f, off);
            fits = P <= G::PREG;
        }
        const bool empty = nA <= 0 || ncols <= 0 || (fits && P == 0);
        bool take = false;
        int nnz = 0;
        if (fits && P > 0) {
            row_dispatch<VALS, AVL, T, IP, G>(S, l, f.cnt, off, P, Bj, Bx, [&](const auto& o) {
                take = o.take;
                nnz = o.nnz;
                if (take && lb) {
                    const int64_t it = row - row0;
                    const unsigned long long g = S.lb_gw;   // (all lanes read the same word)
                    base = row_group_prefix(&sa.gpre[it >> 6],
                                            ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(g >> 32)) << 32) |
                                                (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)g),
                                            row_cnt + row0, it & ~(int64_t)(WAVE - 1), sa.spin) +
                           __builtin_amdgcn_readfirstlane((int)S.lb_gsum);
                    const int64_t end = base + nnz;
                    room = (cap <= 0 || end <= cap) && (sizeof(OFF) == 8 || end <= 2147483647LL);
                }
                if (take && VALS && room) row_write(S, l, o, Cj + base, Cx + base, alpha);
            });
        }
        if (!empty && !take) {
            if (count_all && !(fits && P > 0)) nnz = row_count_only<IP>(S, l, a0, nA, Aj, Bp, Bj);
            if (l == 0 && !(flags & ROW_LISTED)) spill[atomicAdd(spill_count, 1)] = (int32_t)row;
        }
        if (MODE == ROW_SYM && l == 0 && (take || empty || count_all)) row_cnt[row] = take || count_all ? nnz : 0;
        wsync();   // the next row reuses this wave's LDS
    };
#pragma unroll
    for (int q = 0; q < RP; ++q)
        if (q < nr) do_row(row0 + it0 + q, a0s[q], (int)(a0s[q + 1] - a0s[q]), fr[q], lb ? gw[q] : 0ull,
                           lb ? gc[q] : 0);
}

}  // namespace spg
