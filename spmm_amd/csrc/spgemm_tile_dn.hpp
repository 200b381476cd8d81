// spgemm_tile_dn.hpp -- lean kernels of the tile path (dense numeric tiles, long-segment
// symbolic tiles).
//
// Ordered accumulation by LDS atomic add.  Two properties of gfx950's LDS, measured on
// MI355X by abtest/lds_fadd_order.hip (4.2M operand pairs incl. denormals, +-0, inf, nan;
// 50,000 wave instructions with 1.4M same-address lane pairs, every trial bit-exact):
//   * ds_add_f64 rounds exactly like v_add_f64 (IEEE round-to-nearest-even, denormals kept);
//   * the lanes of ONE ds_add_f64 that hit the same address are applied in ascending lane
//     order, and the DS instructions of a wave execute in issue order.
// So if the products of an item are laid out in flattened (jj, kk) order -- A entry
// jj ascending, then the entry's B segment -- 64 per instruction, one `ds_add_f64` per
// 64-product chunk performs every C(i,j) sum in scipy's order: two products of the same
// column come from different A entries, the earlier one sits in an earlier chunk or a lower
// lane of the same chunk.  That replaces the owner-tag rounds of k_tile (a ds_min, a read
// back, a read-add-write and a retry loop per chunk) with one fire-and-forget LDS op.  The
// GPU parity tests re-check the property end to end on every run (bit-exact vs the oracle).
#pragma once

#include "spgemm_tile.hpp"

namespace spg {

// LDS atomic add with the ordering property above, used for fp64 and complex128.
// ds_add_f32 has both properties too (abtest/lds_fadd_order.hip Q4/Q5), but on MI355X it
// costs 193 CU-cycles per wave-instruction against ds_add_f64's 26 (abtest/lds_ops.hip,
// profiles/r03_lds_ops.txt), so fp32 and complex64 keep k_tile's owner rounds: lean fp32
// measured 28.4 ms vs k_tile's 8.45 ms numeric at N=8192, rho=0.1 (profiles/r03_ab/).
template <typename T> struct OrderedLdsAdd : std::false_type {};
template <> struct OrderedLdsAdd<double> : std::true_type {};
template <> struct OrderedLdsAdd<cplx<double>> : std::true_type {};

__device__ __forceinline__ void lds_add(double* p, double v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_add(float* p, float v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <typename R> __device__ __forceinline__ void lds_add(cplx<R>* p, cplx<R> v) {
    lds_add(&p->re, v.re);
    lds_add(&p->im, v.im);
}

// Run-time check of the two properties above (spg_create, lds_order_check in spgemm.hip):
// LDSCHK_TRIALS trials; in each, two ds_add_f64 (ds_add_f32) instructions from all 64 lanes into 4
// slots (v and slot indexed [trial][instruction][lane]); the slots' sums go to out[trial][4].
constexpr int LDSCHK_TRIALS = 64;
template <typename T>
__global__ __launch_bounds__(WAVE) void k_lds_order_check(const T* __restrict__ v, const int* __restrict__ slot,
                                                          T* __restrict__ out) {
    __shared__ T acc[4];
    const int l = lane_id();
    for (int t = 0; t < LDSCHK_TRIALS; ++t) {
        if (l < 4) acc[l] = (T)0;
        wsync();
        const int i0 = t * 2 * WAVE + l, i1 = i0 + WAVE;
        const T v0 = v[i0], v1 = v[i1];
        const int s0 = slot[i0], s1 = slot[i1];
        lds_add(&acc[s0], v0);
        lds_add(&acc[s1], v1);
        wsync();
        if (l < 4) out[t * 4 + l] = acc[l];
        wsync();
    }
}

// C's stores and the streamed per-item reads (A rows, item offsets) with or without the
// non-temporal hint (SPG_NT_C / SPG_NT_A, A/B builds), so they do not push the tile's B
// slice out of the XCD's L2.
#ifndef SPG_NT_C
#define SPG_NT_C 1
#endif
// SPG_NT_A: non-temporal A-row reads in the dense-tile kernel (1, default: config 4 19.8 -> 19.4 ms;
// the sparse-tile kernel keeps plain loads, config 5 98.7 -> 100.5 ms with them; 2: both)
#ifndef SPG_NT_A
#define SPG_NT_A 1
#endif
// SPG_NT_C: 1 non-temporal (`nt`), 0 plain, 2 agent-scope (`sc1`), 3 system-scope (`sc0 sc1`)
// stores; A/B builds only: 4 `sc1 nt`, 5 `sc0 nt`, 6 `sc0` (vector stores in inline asm)
#define SPG_ST_ASM(POL)                                                                               \
    if constexpr (sizeof(T) == 8) asm volatile("global_store_dwordx2 %0, %1, off " POL ::"v"(p), "v"(v) : "memory"); \
    else asm volatile("global_store_dword %0, %1, off " POL ::"v"(p), "v"(v) : "memory");
template <typename T> __device__ __forceinline__ void st_c(T* p, T v) {
    if constexpr (SPG_NT_C >= 4 && (sizeof(T) == 4 || sizeof(T) == 8)) {
        if constexpr (SPG_NT_C == 4) { SPG_ST_ASM("sc1 nt") }
        else if constexpr (SPG_NT_C == 5) { SPG_ST_ASM("sc0 nt") }
        else { SPG_ST_ASM("sc0") }
    } else if constexpr (SPG_NT_C == 2 && (sizeof(T) == 4 || sizeof(T) == 8))
        __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if constexpr (SPG_NT_C == 3 && (sizeof(T) == 4 || sizeof(T) == 8))
        __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else if constexpr (SPG_NT_C != 0 && (sizeof(T) == 4 || sizeof(T) == 8)) __builtin_nontemporal_store(v, p);
    else *p = v;
}
template <typename R> __device__ __forceinline__ void st_c(cplx<R>* p, cplx<R> v) {
    st_c(&p->re, v.re);
    st_c(&p->im, v.im);
}
template <bool NT = (SPG_NT_A != 0), typename T> __device__ __forceinline__ T ld_a(const T* p) {
    if constexpr (NT && (sizeof(T) == 4 || sizeof(T) == 8)) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT = (SPG_NT_A != 0), typename R> __device__ __forceinline__ cplx<R> ld_a(const cplx<R>* p) {
    return cplx<R>(ld_a<NT>(&p->re), ld_a<NT>(&p->im));
}
constexpr bool SP_NT_A = SPG_NT_A == 2;   // (the sparse-tile kernels)

constexpr int DN_WPB = 2;     // waves per block
#ifndef SPG_RG_SYNC
#define SPG_RG_SYNC 1   // items between the barriers of a cooperative record-group block
#endif

// Per-batch A-entry table: the byte offset of the entry's first product record, shifted by
// the entry's flattened offset (so product t of the batch reads base[src] + t * RB), and the
// A value.  One 16-byte LDS read per product lane (f64).  Entry WAVE is the batch's pseudo
// entry: from product Pb on (past the batch's products, up to the end of the step) the slots
// read the sentinel records (spgemm_tile.hpp), which add 0 into slots nobody reads -- no
// compare, select or clamp per chunk.
template <typename T> struct __attribute__((aligned(16))) DnEnt {
    uint32_t base;
    uint32_t pad;
    T a;
};


// fp64 items take their structure from the accumulator itself (SPG_DN_SENT): every slot
// starts at -0.0 instead of +0.0.  -0.0 + p == +0.0 + p for every p except p == -0.0, so a
// column's sum equals scipy's (which starts at +0.0) except while every product it has seen
// is -0.0 (ours -0.0, scipy's +0.0).  So a column is reached iff its slot is not -0.0 or it
// saw only -0.0 products; the item's symbolic count tells which case holds: fewer non -0.0
// slots than entries sends the item down a rare path that re-walks its products and turns
// each reached -0.0 slot into scipy's +0.0.  No hit byte per product.
#ifndef SPG_DN_SENT
#define SPG_DN_SENT 1
#endif
template <typename T> constexpr bool dn_sent() {
    return SPG_DN_SENT && (std::is_same<T, double>::value || std::is_same<T, float>::value);
}
// the -0.0 sentinel's bits and the bits of a real value
template <typename T> __device__ __forceinline__ bool is_neg_zero(T v) {
    if constexpr (sizeof(T) == 8) return __double_as_longlong(v) == (long long)0x8000000000000000ull;
    else return __float_as_uint(v) == 0x80000000u;
}

// Chunks (64 products) per marker group of the ordered walk (dn_walk), all of a group's
// record loads in flight together: 16 for the widest kernels (2048-slot accumulators: LDS
// holds them to 2 waves per SIMD, so the extra registers are free; round 4, config 4
// numeric -2 %, config 5 -1 %), 8 for the 1024-slot ones (4 waves per SIMD at <= 128 VGPRs).
#ifndef SPG_DN_U16
#define SPG_DN_U16 1
#endif
__host__ __device__ constexpr int dn_mkb(int slots) { return (SPG_DN_U16 && slots >= 2048) ? 16 : 8; }

template <typename T, int TWD, bool HIT = !dn_sent<T>()> struct DnLds {
    T acc[TWD + DN_DUMMY];        // accumulator by column; + the sentinel records' slots
    DnEnt<T> ent[WAVE + 1];
    uint8_t mk[dn_mkb(TWD) * WAVE];   // lane -> A-entry markers of one group's chunks
    uint8_t hit[TWD + DN_DUMMY];  // columns some product reached (non-sentinel types)
};
// (dn_sent, TWD 1024: 10,000 bytes per wave -- 8 two-wave blocks, 16 waves, fit a CU's 160 KB;
// TWD 2048: 18,192 bytes, 8 waves)
template <typename T, int TWD> struct DnLds<T, TWD, false> {
    T acc[TWD + DN_DUMMY];
    DnEnt<T> ent[WAVE + 1];
    uint8_t mk[dn_mkb(TWD) * WAVE];
#ifdef SPG_LDS_PAD
    uint8_t pad[SPG_LDS_PAD];   // (A/B builds: occupancy sensitivity)
#endif
};


// Markers of one group of 8 chunks (transposed as num_group_markers): entry l's first product
// gets l + 1, and product Pb (the batch's end, if inside the group) the pseudo entry's WAVE + 1.
template <int MKB>
__device__ __forceinline__ void dn_group_markers(uint8_t* mk, int l, int cnt, int off, int gb, int Pb) {
    constexpr int SH = MKB == 16 ? 4 : 3;
    constexpr int DN_MK = MKB * WAVE;
    wsync();
    if constexpr (MKB == 16) reinterpret_cast<uint4*>(mk)[l] = make_uint4(0u, 0u, 0u, 0u);
    else reinterpret_cast<uint2*>(mk)[l] = make_uint2(0u, 0u);
    wsync();
    if (cnt > 0 && off >= gb && off < gb + DN_MK) {
        const int t = off - gb;
        mk[((t & (WAVE - 1)) << SH) | (t >> 6)] = (uint8_t)(l + 1);
    }
    if (l == 0 && Pb - gb < DN_MK) {
        const int t = Pb - gb;
        mk[((t & (WAVE - 1)) << SH) | (t >> 6)] = (uint8_t)(WAVE + 1);
    }
    wsync();
}

// One batch of up to 64 A entries of the ordered walk (lane l: entry b + l, segment length
// `cnt` at byte offset `bb` of the record array, A value `av`): the DPP scan of the segment
// lengths and the entry table in LDS; per group of MKB chunks the transposed markers; per U
// chunks the lane -> entry max-scans, one 16-byte table read and one record load per chunk (all
// in flight), then per chunk in order one multiply and one ds_add_f64 into acc[slot(column)]
// and hit(slot).  `sent` is the byte offset of the kernel's sentinel region.
template <typename T, int MKB, typename L, typename Slot, typename Hit>
__device__ __forceinline__ void dn_batch(L* lp, T* acc, int l, int cnt, uint32_t bb, T av, const char* __restrict__ rb,
                                         uint32_t sent, Slot&& slot, Hit&& hit) {
    constexpr int U = (sizeof(T) > 8 ? 4 : 8) * (MKB / 8);   // chunks in flight
    constexpr int DN_MK = MKB * WAVE;                         // products per marker group
    constexpr uint32_t RB = (uint32_t)rec_bytes<T>();   // bytes of one B record
    DnEnt<T>* ent = lp->ent;
    uint8_t* mk = lp->mk;
    const int incl = wave_incl_sum_dpp(cnt);
    const int off = incl - cnt;
    const int Pb = readlane_i(incl, WAVE - 1);
    wsync();
    ent[l].base = bb - (uint32_t)off * RB;   // wraps; base + t*RB is exact
    ent[l].a = av;
    if (l == 0) {
        ent[WAVE].base = sent - (uint32_t)Pb * RB;   // products Pb.. read sentinel records
        ent[WAVE].a = (T)0;
    }
    unsigned carry = 0u;
    for (int gb = 0; gb < Pb; gb += DN_MK) {
        dn_group_markers<MKB>(mk, l, cnt, off, gb, Pb);
        const int nchg = min(DN_MK, Pb - gb);
        uint64_t mrow[MKB / 8];   // this lane's marker byte of each chunk of the group
        if constexpr (MKB == 16) {
            const uint4 m4 = reinterpret_cast<const uint4*>(mk)[l];
            mrow[0] = ((uint64_t)m4.y << 32) | m4.x;
            mrow[(MKB / 8) - 1] = ((uint64_t)m4.w << 32) | m4.z;
        } else {
            const uint2 m2 = reinterpret_cast<const uint2*>(mk)[l];
            mrow[0] = ((uint64_t)m2.y << 32) | m2.x;
        }
        for (int c0 = 0; c0 < nchg; c0 += U * WAVE) {
            const int nu = min(U, (nchg - c0 + WAVE - 1) >> 6);
            auto step = [&](auto nuc) {
                constexpr int NU = decltype(nuc)::value;
                const int cb = c0 >> 6;   // first chunk of the step (0 when U covers the group)
                unsigned sp[NU];
#pragma unroll
                for (int u = 0; u < NU; ++u) {
                    const int i = cb + u;
                    const uint64_t w = (MKB == 16 && i >= 8) ? mrow[(MKB / 8) - 1] : mrow[0];
                    sp[u] = wave_incl_umax_dpp((unsigned)(w >> (8 * (i & 7))) & 0xffu);
                }
#pragma unroll
                for (int u = 0; u < NU; ++u) {
                    sp[u] = max(sp[u], carry);
                    carry = (unsigned)readlane_i((int)sp[u], WAVE - 1);
                }
                // product 0 of a batch always carries a marker, so sp >= 1; slots past the
                // batch's products carry the pseudo entry's
                int qc[NU];
                T qv[NU], qa[NU];
#pragma unroll
                for (int u = 0; u < NU; ++u) {
                    const uint32_t t = (uint32_t)(gb + c0 + u * WAVE + l);
                    uint32_t eb;
                    if constexpr (sizeof(T) <= 8) {   // base and value with one 16-byte read
                        const uint4 e4 = reinterpret_cast<const uint4*>(ent)[(int)sp[u] - 1];
                        eb = e4.x;
                        const uint32_t w2[2] = {e4.z, e4.w};
                        __builtin_memcpy(&qa[u], w2, sizeof(T));
                    } else {
                        const DnEnt<T> e = ent[(int)sp[u] - 1];
                        eb = e.base;
                        qa[u] = e.a;
                    }
                    if constexpr ((SPG_TILE_DIAG & 2) != 0) {   // timing only: no record loads
                        qc[u] = (int)(((eb + t * 2654435761u) >> 22) & 1023u);
                        qv[u] = (T)1;
                    } else {
                        load_rec_at(rb, eb + __umul24(t, RB), qc[u], qv[u]);
                    }
                }
#pragma unroll
                for (int u = 0; u < NU; ++u) {
                    const int c = slot(qc[u]);
                    if constexpr ((SPG_TILE_DIAG & 16) != 0) {   // timing only: plain LDS stores
                        acc[c] = mul_rn(qa[u], qv[u]);
                    } else if constexpr ((SPG_TILE_DIAG & 32) != 0) {   // timing only: conflict-free adds
                        lds_add(&acc[l + (c & 1)], mul_rn(qa[u], qv[u]));
                    } else if constexpr ((SPG_TILE_DIAG & 1) == 0 && OrderedLdsAdd<T>::value) {   // (diag 1: none)
                        lds_add(&acc[c], mul_rn(qa[u], qv[u]));   // chunk order = issue order
                        hit(c);
                    } else if constexpr ((SPG_TILE_DIAG & 1) == 0) {
                        // fp32 (round 5): ds_add_f32 costs 193 CU-cycles per wave instruction on
                        // MI355X, a plain read-add-write 17.  The products of ONE A entry in a
                        // chunk hit distinct columns (a B row's columns are distinct), so the
                        // chunk's run of each entry (sp[u], non-decreasing over the lanes) adds
                        // with a plain read-add-write, runs in entry order; a chunk holding more
                        // than two entries adds its third and later runs with one ordered
                        // ds_add_f32 (ascending lanes = entry order).  Lanes past the batch
                        // (pseudo entry) add nothing.
                        const T pv = mul_rn(qa[u], qv[u]);
                        bool live = sp[u] <= (unsigned)WAVE;
                        // two runs whose column ranges do not overlap (a segment's tail in
                        // high columns, the next segment's head in low ones -- most chunks
                        // that hold a segment boundary) are distinct too: one read-add-write
                        const unsigned long long lm = __ballot(live);   // live lanes: a prefix
                        if (lm != 0ull) {
                            const unsigned e0 = (unsigned)readlane_i((int)sp[u], 0);
                            const unsigned long long m2 = __ballot(live && sp[u] != e0);
                            bool one = m2 == 0ull;
                            if (!one) {
                                const int l2 = (int)__builtin_ctzll(m2), last = 63 - (int)__builtin_clzll(lm);
                                const unsigned e1 = (unsigned)readlane_i((int)sp[u], l2);
                                if (__ballot(live && sp[u] != e0 && sp[u] != e1) == 0ull) {
                                    const int c1 = readlane_i(c, 0), ck = readlane_i(c, l2 - 1);
                                    const int d1 = readlane_i(c, l2), dm = readlane_i(c, last);
                                    one = dm < c1 || d1 > ck;
                                }
                            }
                            if (one) {
                                if (live) acc[c] = add_rn(acc[c], pv);
                                live = false;
                            }
                        }
                        for (int run = 0;; ++run) {
                            const unsigned long long m = __ballot(live);
                            if (m == 0ull) break;
                            if (run == 2) {
                                if (live) lds_add(&acc[c], pv);
                                break;
                            }
                            const unsigned e0 = (unsigned)readlane_i((int)sp[u], (int)__builtin_ctzll(m));
                            if (live && sp[u] == e0) {
                                acc[c] = add_rn(acc[c], pv);
                                live = false;
                            }
                            wsync();   // (fence + barrier: no LDS access moves across a run boundary)
                        }
                        hit(c);
                    }
                }
            };
            if (nu > 3 * U / 4) step(std::integral_constant<int, U>{});
            else if (nu > U / 2) step(std::integral_constant<int, 3 * U / 4>{});
            else if (nu > U / 4) step(std::integral_constant<int, U / 2>{});
            else step(std::integral_constant<int, U / 4>{});
        }
    }
}

// Batch b's entries (the first NB batches from the register queue `sq`/`aq`, the rest loaded).
template <typename T, int NB>
__device__ __forceinline__ void dn_fetch(int b, int l, const int32_t* __restrict__ tp, int64_t a0, int nA, T (&aq)[NB],
                                         uint2 (&sq)[NB], const int32_t* __restrict__ Aj, const T* __restrict__ Ax,
                                         int rgs, int& cnt, uint32_t& bb, T& av) {
    constexpr uint32_t RB = (uint32_t)rec_bytes<T>();
    cnt = 0;
    bb = 0;   // byte offset of the entry's segment in the record array
    av = (T)0;
    if (b < NB * WAVE) {
        // the preloaded batches queue in registers: take the head, shift the rest down
        // (static register indices: a select chain or a dynamic index costs more)
        cnt = (int)(sq[0].y - sq[0].x);
        bb = sq[0].x * RB;
        av = aq[0];
#pragma unroll
        for (int q = 0; q + 1 < NB; ++q) {
            sq[q] = sq[q + 1];
            aq[q] = aq[q + 1];
        }
    } else if (b + l < nA) {
        const uint2 se = seg_pair(tp, Aj[a0 + b + l], rgs);
        cnt = (int)(se.y - se.x);
        bb = se.x * RB;
        av = Ax[a0 + b + l];
    }
}

// The ordered product walk of one item (row, tile): its A entries in batches of 64 (the first
// NB batches' tile segments `sq` and values `aq` given, the rest loaded here), one dn_batch each.
template <typename T, int NB, int MKB, typename L, typename Slot, typename Hit>
__device__ __forceinline__ void dn_walk(L* lp, T* acc, int l, const int32_t* __restrict__ tp, int64_t a0, int nA,
                                        T (&aq)[NB], uint2 (&sq)[NB], const int32_t* __restrict__ Aj,
                                        const T* __restrict__ Ax, const char* __restrict__ rb, uint32_t sent,
                                        int rgs, Slot&& slot, Hit&& hit) {
    for (int b = 0; b < nA; b += WAVE) {
        int cnt;
        uint32_t bb;
        T av;
        dn_fetch<T, NB>(b, l, tp, a0, nA, aq, sq, Aj, Ax, rgs, cnt, bb, av);
        dn_batch<T, MKB>(lp, acc, l, cnt, bb, av, rb, sent, slot, hit);
    }
}

// The item's output: its structure 64 columns at a time from hit[] or (dn_sent) the slots that
// left -0.0 (ballot + lane rank give positions), straight to C; the rare -0.0 re-walk.
template <typename T, int TWD>
__device__ __forceinline__ void dn_emit(DnLds<T, TWD>& S, int l, int TW, int lo, int nnz, const int32_t* __restrict__ tp,
                                        int64_t a0, int nA, const int32_t* __restrict__ Aj,
                                        const char* __restrict__ rb, int32_t* __restrict__ crow,
                                        T* __restrict__ xrow, T alpha, int rgs, int32_t* cj0 = nullptr,
                                        T* cx0 = nullptr) {
    constexpr uint32_t RB = (uint32_t)rec_bytes<T>();
    // (diag 1024, timing only: every store full and aligned, into a per-wave 64-entry region of C)
    const uint32_t wreg = ((blockIdx.x * DN_WPB + (threadIdx.x >> 6)) & 4095u) * 64u;
    int32_t* crow_al = cj0 + wreg;
    T* xrow_al = cx0 + wreg;
    wsync();
    // the item's structure, 64 columns at a time: hit[] or (dn_sent) the non -0.0 slots
    // (4 column groups per round: their LDS reads in flight together, TW >= 256)
    auto emit = [&](auto one) {
        int run = 0;
        for (int k0 = 0; k0 < TW / WAVE; k0 += 4) {
            T v[4];
            bool h[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int c = (k0 + e) * WAVE + l;
                v[e] = S.acc[c];
                if constexpr (dn_sent<T>()) h[e] = !is_neg_zero(v[e]);
                else h[e] = S.hit[c] != 0;
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const unsigned long long m = __ballot(h[e]);
                if constexpr ((SPG_TILE_DIAG & 1024) != 0) {   // (diag 1024: full aligned 64-lane stores)
                    st_c(crow_al + l, (int32_t)(lo + (k0 + e) * WAVE + l));
                    st_c(xrow_al + l, v[e]);
                } else if (h[e] && (SPG_TILE_DIAG & 8) == 0) {   // (diag 8, timing only: no output)
                    uint32_t p = (uint32_t)(run + lane_rank(m));
                    if constexpr ((SPG_TILE_DIAG & 128) != 0) p &= 63u;   // (diag 128: the same stores, L2-resident)
                    st_c(crow + p, (int32_t)(lo + (k0 + e) * WAVE + l));
                    st_c(xrow + p, decltype(one)::value ? v[e] : mul_rn(alpha, v[e]));
                }
                run += (int)__popcll(m);
            }
        }
        return run;
    };
    const bool one = alpha == (T)1;
    const int got = one ? emit(std::true_type{}) : emit(std::false_type{});
    if constexpr (dn_sent<T>()) {
        if (got < nnz && (SPG_TILE_DIAG & 9) == 0) {
            // rare: a reached column saw only -0.0 products -- its slot is still -0.0, scipy's
            // sum is +0.0.  Re-walk the item's records (one lane per A entry) and turn every
            // reached -0.0 slot into +0.0, then write the item again.
            for (int b = 0; b < nA; b += WAVE) {
                if (b + l < nA) {
                    const uint2 se = seg_pair(tp, Aj[a0 + b + l], rgs);
                    for (uint32_t i = se.x; i < se.y; ++i) {
                        int c;
                        T v;
                        load_rec(reinterpret_cast<const uint32_t*>(rb + (uint64_t)i * RB), 0, c, v);
                        if (is_neg_zero(S.acc[c])) S.acc[c] = (T)0;
                    }
                }
            }
            wsync();
            if (one) emit(std::true_type{});
            else emit(std::false_type{});
        }
    }
}

// clear an item's accumulator
template <typename T, int TWD>
__device__ __forceinline__ void dn_clear(DnLds<T, TWD>& S, int l, int TW) {
    wsync();
    // clear the accumulator (-0.0: dn_sent) and the hit bytes (16-byte stores; TW is a
    // multiple of 64)
    uint4* a4 = reinterpret_cast<uint4*>(S.acc);
    const uint32_t hi = dn_sent<T>() ? 0x80000000u : 0u;       // -0.0's sign bit
    const uint32_t lw = sizeof(T) == 4 ? hi : 0u;              // (fp32: every word is a value)
    for (int q = l; q < TW * (int)sizeof(T) / 16; q += WAVE) a4[q] = make_uint4(lw, hi, lw, hi);
    if constexpr (!dn_sent<T>()) {
        uint4* h4 = reinterpret_cast<uint4*>(S.hit);
        for (int q = l; q < TW / 16; q += WAVE) h4[q] = make_uint4(0u, 0u, 0u, 0u);
    }
}

// One dense-tile item (row, tile g of TW <= TWD columns) on one wave: clear the accumulator,
// the ordered product walk with slot = column, then the output.
template <typename T, int NB, int TWD>
__device__ __forceinline__ void dn_item(DnLds<T, TWD>& S, int l, int TW, int lo, int nnz, const int32_t* __restrict__ tp,
                                        int64_t a0, int nA, T (&aq)[NB], uint2 (&sq)[NB],
                                        const int32_t* __restrict__ Aj,
                                        const T* __restrict__ Ax, const char* __restrict__ rb, uint32_t sent,
                                        int32_t* __restrict__ crow,
                                        T* __restrict__ xrow, T alpha, int rgs, int32_t* cj0, T* cx0) {
    dn_clear(S, l, TW);
    dn_walk<T, NB, dn_mkb(TWD)>(&S, S.acc, l, tp, a0, nA, aq, sq, Aj, Ax, rb, sent, rgs, [&](int c) { return c; },
                   [&](int c) {
                       if constexpr (!dn_sent<T>()) S.hit[c] = 1;
                   });
    dn_emit<T, TWD>(S, l, TW, lo, nnz, tp, a0, nA, Aj, rb, crow, xrow, alpha, rgs, cj0, cx0);
}
// Numeric pass on dense tiles: one wave per (row, tile) item, items tile-major over the
// XCD-aware block map (an XCD works through one tile at a time, so the tile's B slice and
// segment table stay in its L2), the first NB batches' A entries and tile segments loaded up
// front.
// RG = 1: the two waves of a block take independent items (tile-major).  RG = DN_WPB (A/B
// builds, SPG_DN_RGS): the block's two waves take the two tiles of one record group of the same
// row (items group-major), starting together every SPG_RG_SYNC items, as k_tile_sp<.., RG>.
template <typename T, typename IP, int TWD, int RG = 1>
__global__ __launch_bounds__(DN_WPB * WAVE) void k_tile_dn(
    int64_t row0, int64_t nrows, int tws, int G, const IP* __restrict__ Ap,
    const int32_t* __restrict__ Aj, const T* __restrict__ Ax, int64_t K,
    const uint32_t* __restrict__ brec, const int32_t* __restrict__ tptr,
    const int64_t* __restrict__ item_off, int32_t* __restrict__ Cj, T* __restrict__ Cx, T alpha, uint32_t sent,
    uint32_t it_lo, uint32_t it_hi, int rgs) {
    static_assert(RG == 1 || RG == DN_WPB, "a record group is the block's waves");
    static_assert(OrderedLdsAdd<T>::value || std::is_same<T, float>::value, "ordered LDS add or fp32 runs");
    constexpr int NB = sizeof(T) > 8 ? 4 : 8;    // A batches preloaded per item
    __shared__ __attribute__((aligned(16))) DnLds<T, TWD> lds[DN_WPB];
    const int l = lane_id();
    const int wv = uniform((int)(threadIdx.x >> 6));
    DnLds<T, TWD>& S = lds[wv];
    const int TW = 1 << tws;
    const char* __restrict__ rb = reinterpret_cast<const char*>(brec);
    // items [it_lo, it_hi) (tile-major: a range of whole tiles; rows*G < 2^31 on the host;
    // RG > 1: (record group, row) items, one per block)
    constexpr uint32_t PER = RG > 1 ? 1u : (uint32_t)DN_WPB;
    uint32_t sweep = 0;
    for (uint32_t it = it_lo + xcd_block(gridDim.x) * PER + (RG > 1 ? 0u : (uint32_t)wv); it < it_hi;
         it += gridDim.x * PER, ++sweep) {
        if constexpr (RG > 1) {
            if (sweep % SPG_RG_SYNC == 0) __syncthreads();
        }
        const int grp = (int)(it / (uint32_t)nrows);
        const int64_t row = row0 + (int64_t)(it - (uint32_t)grp * (uint32_t)nrows);
        const int g = RG > 1 ? grp * RG + wv : grp;
        if (RG > 1 && g >= G) continue;   // (a padding tile of the last group)
        const int64_t item = (row - row0) * G + g;
        const int64_t obase = ld_a(item_off + item);
        const int nnz = (int)(ld_a(item_off + item + 1) - obase);
        if (nnz == 0) continue;                      // (no product reaches this tile)
        const int32_t* __restrict__ tp = tptr + tile_table_off(g, K, rgs);
        const int64_t a0 = Ap[row];
        const int nA = (int)(Ap[row + 1] - a0);
        int32_t kq[NB];
        T aq[NB];
        uint2 sq[NB];
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            kq[q] = -1;
            aq[q] = (T)0;
            if (q * WAVE + l < nA) {
                kq[q] = ld_a(Aj + a0 + q * WAVE + l);
                aq[q] = ld_a(Ax + a0 + q * WAVE + l);
            }
        }
#pragma unroll
        for (int q = 0; q < NB; ++q) sq[q] = kq[q] >= 0 ? seg_pair(tp, kq[q], rgs) : make_uint2(0u, 0u);
        dn_item<T, NB, TWD>(S, l, TW, g * TW, nnz, tp, a0, nA, aq, sq, Aj, Ax, rb, sent, Cj + obase, Cx + obase, alpha,
                            rgs, Cj, Cx);
    }
}

// ---------------------------------------------------------------------------------------
// Numeric pass on sparse tiles (TW up to 4096 columns, config 5's shape): the item's structure
// is its symbolic bitmap; the accumulator is compact -- a product's slot is its column's rank
// among the item's columns (the bitmap word's popcount prefix plus the bits below it) -- in
// windows of at most TILE_CAP slots (an item with more entries re-walks its products once
// per window).  The same ordered walk as the dense tiles (one ds_add_f64 per 64 products).
// Output per window: the compact accumulator is already in C order, so the values leave with
// coalesced stores; then every lane lists its bitmap words' columns (one per set bit) into the
// freed accumulator, and the column indices leave the same way.
// The kernel is instantiated for two tile widths: up to 4096 columns (1024-slot windows, 128
// bitmap words) and, fp64 only, 8192 columns (2048-slot windows, 256 words: config 5's
// shape, numeric 128.7 -> 103.9 ms; 16384 columns measured 143 ms with 2048-slot windows and,
// round 4, 138 ms with one 4096-slot window: 39 KB of LDS per wave leaves 4 waves per CU).
// LDS geometry of a sparse-tile kernel: CAP window slots, NW bitmap words (TW <= 32 * NW
// columns), DUMMY lane slots past the window (the out-of-window and sentinel products add
// there: lane l into CAP + (l % DUMMY)), MKB chunks per marker group.
template <int CAP_, int NW_, int DUMMY_, int MKB_> struct SpCfg {
    static constexpr int CAP = CAP_, NW = NW_, DUMMY = DUMMY_, MKB = MKB_;
    static constexpr int WPL = NW / WAVE;          // bitmap words per lane (at most)
};
using SpCfg1024 = SpCfg<1024, 128, WAVE, 8>;    // tiles of <= 4096 columns (11.3 KB per wave)
using SpCfg2048 = SpCfg<2048, 256, WAVE, 16>;   // fp64 8192-column tiles (21.0 KB)
// fp64 8192-column tiles in cooperative blocks of RG waves (k_tile_sp<.., RG>, A/B builds with
// SPG_SP_RGS > 0): 20,432 bytes per wave, so two 4-wave blocks (8 waves) fit a CU's 160 KB;
// 2032 slots per window (config 5's items hold 1887 +- 40 entries) and 8 lane slots (an
// out-of-window add conflicts at most 8 ways)
#ifndef SPG_RG_MKB
#define SPG_RG_MKB 16   // (A/B: chunks per marker group of the cooperative kernel)
#endif
using SpCfgRG = SpCfg<2032, 256, 8, SPG_RG_MKB>;
template <typename T, typename CF> struct SpLds {
    T acc[CF::CAP + CF::DUMMY];         // compact accumulator of one window; + lane slots
    uint2 bw[CF::NW];                   // (bitmap word, popcount prefix)
    DnEnt<T> ent[WAVE + 1];
    uint8_t mk[CF::MKB * WAVE];
#ifdef SPG_LDS_PAD
    uint8_t pad[SPG_LDS_PAD];   // (A/B builds: occupancy sensitivity)
#endif
};

// RG = 1: one-wave blocks, items tile-major (item it = (tile, row)).
// RG > 1 (cooperative record groups, round 5): blocks of RG waves, items group-major (it =
// (group, row)); wave t of the block takes tile group*RG + t of the same row.  The RG tiles'
// segments of one B row are adjacent in the record-group layout (k_bt_pack), so the block's
// waves walk one contiguous run of records per A entry instead of RG separate ~80-byte
// segments in RG slices: config 5's segments are 8 records (82 bytes) per 8192-column tile,
// and a lone segment costs 1.6 128-byte lines.  A barrier at every item keeps the waves on
// the same A entries, so the lines they share are fetched once.  The accumulation is per
// wave and per tile, exactly as with RG = 1 (same results bit for bit).
template <typename T, typename IP, typename CF, int RG>
__global__ __launch_bounds__(RG * WAVE) __attribute__((amdgpu_waves_per_eu((sizeof(T) > 8 || CF::CAP > 1024) ? 2 : 4)))
void k_tile_sp(
    int64_t row0, int64_t nrows, int tws, int G, const IP* __restrict__ Ap,
    const int32_t* __restrict__ Aj, const T* __restrict__ Ax, int64_t K,
    const uint32_t* __restrict__ brec, const int32_t* __restrict__ tptr, const uint32_t* __restrict__ bitmap,
    const int64_t* __restrict__ item_off, int32_t* __restrict__ Cj, T* __restrict__ Cx, T alpha, uint32_t sent,
    uint32_t it_lo, uint32_t it_hi, int rgs) {
    static_assert(OrderedLdsAdd<T>::value, "ordered LDS add needed");
    constexpr int SP_CAP = CF::CAP;
    constexpr int SP_DUMMY = CF::DUMMY;
    static_assert((SP_DUMMY & (SP_DUMMY - 1)) == 0, "lane slots: a power of two");
    static_assert(sizeof(T) * (SP_CAP + SP_DUMMY) >= 4 * SP_CAP, "column list fits the accumulator");
    constexpr int SP_WPL = CF::WPL;
    constexpr int NB = sizeof(T) > 8 ? 4 : 8;
    __shared__ __attribute__((aligned(16))) SpLds<T, CF> lds[RG];
    const int l = lane_id();
    const int wv = uniform((int)(threadIdx.x >> 6));
    SpLds<T, CF>& S = lds[wv];
    const int TW = 1 << tws;
    const int nw = TW >> 5;                    // bitmap words of a tile
    const int wpl = (nw + WAVE - 1) / WAVE;    // words per lane (<= SP_WPL)
    const char* __restrict__ rb = reinterpret_cast<const char*>(brec);
    const bool one = alpha == (T)1;
    // one item per block and sweep (RG == 1: a one-wave block's; RG > 1: the group's RG tiles of a row)
    uint32_t sweep = 0;
    for (uint32_t it = it_lo + xcd_block(gridDim.x); it < it_hi; it += gridDim.x, ++sweep) {
        // RG > 1: the block's waves start together every SPG_RG_SYNC items (a persistent grid:
        // between two barriers a wave that finishes early starts its next item)
        if constexpr (RG > 1) {
            if (sweep % SPG_RG_SYNC == 0) __syncthreads();
        }
        const int grp = (int)(it / (uint32_t)nrows);
        const int64_t row = row0 + (int64_t)(it - (uint32_t)grp * (uint32_t)nrows);
        const int g = RG == 1 ? grp : grp * RG + wv;
        if (RG > 1 && g >= G) continue;           // (a padding tile of the last group)
        const int64_t item = (row - row0) * G + g;
        const int32_t* __restrict__ tp = tptr + tile_table_off(g, K, rgs);
        const int64_t a0 = Ap[row];
        const int nA = (int)(Ap[row + 1] - a0);
        if (nA <= 0) continue;
        // the item's bitmap (lane owns wpl words) and its popcount prefix
        const uint32_t* __restrict__ ibits = bitmap + item * nw;
        const int w0 = min(nw, l * wpl), w1 = min(nw, w0 + wpl);
        uint32_t wd[SP_WPL] = {};
        int mine = 0;
        if (SP_WPL % 4 == 0 && wpl == SP_WPL) {   // (widest tiles: a lane's words in 16-byte loads)
#pragma unroll
            for (int h = 0; h < SP_WPL / 4; ++h) {
                const uint4 w4 = *reinterpret_cast<const uint4*>(ibits + w0 + 4 * h);
                wd[(4 * h) % SP_WPL] = w4.x;
                wd[(4 * h + 1) % SP_WPL] = w4.y;
                wd[(4 * h + 2) % SP_WPL] = w4.z;
                wd[(4 * h + 3) % SP_WPL] = w4.w;
            }
#pragma unroll
            for (int q = 0; q < SP_WPL; ++q) mine += __popc(wd[q]);
        } else {
#pragma unroll
            for (int q = 0; q < SP_WPL; ++q)
                if (w0 + q < w1) {
                    wd[q] = ibits[w0 + q];
                    mine += __popc(wd[q]);
                }
        }
        const int pincl = wave_incl_sum_dpp(mine);
        const int nnz = readlane_i(pincl, WAVE - 1);
        if (nnz == 0) continue;
        const int p0 = pincl - mine;
        T aq[NB];
        uint2 sq[NB];
        auto preload = [&]() {
            int32_t kq[NB];
#pragma unroll
            for (int q = 0; q < NB; ++q) {
                kq[q] = -1;
                aq[q] = (T)0;
                if (q * WAVE + l < nA) {
                    kq[q] = ld_a<SP_NT_A>(Aj + a0 + q * WAVE + l);
                    aq[q] = ld_a<SP_NT_A>(Ax + a0 + q * WAVE + l);
                }
            }
#pragma unroll
            for (int q = 0; q < NB; ++q) sq[q] = kq[q] >= 0 ? seg_pair(tp, kq[q], rgs) : make_uint2(0u, 0u);
        };
        preload();
        const int64_t obase = item_off[item];
        wsync();
        {
            int run = p0;
#pragma unroll
            for (int q = 0; q < SP_WPL; ++q)
                if (w0 + q < w1) {
                    S.bw[w0 + q] = make_uint2(wd[q], (uint32_t)run);
                    run += __popc(wd[q]);
                }
        }
        const int lo = g * TW;
        for (int L0 = 0; L0 < WAVE;) {
            // window: lanes [L0, L1) whose words' entries fit SP_CAP slots
            int L1 = WAVE, wb = 0, wn = nnz;
            if (nnz > SP_CAP) {
                wb = readlane_i(p0, L0);
                L1 = (int)__popcll(__ballot(pincl <= wb + SP_CAP));
                if (L1 <= L0) L1 = L0 + 1;
                wn = (L1 < WAVE ? readlane_i(p0, L1) : nnz) - wb;
            }
            const int clo = 32 * wpl * L0, chi = 32 * wpl * L1;   // window, tile-relative
            wsync();
            for (int p = l; p < wn; p += WAVE) S.acc[p] = (T)0;
            if (L0 > 0) preload();   // (the walk consumes the queue; rare later windows reload it)
            dn_walk<T, NB, CF::MKB>(&S, S.acc, l, tp, a0, nA, aq, sq, Aj, Ax, rb, sent, rgs,
                           [&](int rc) -> int {
                               if (rc < clo || rc >= chi) return SP_CAP + (l & (SP_DUMMY - 1));   // (sentinels too)
                               const uint2 b = S.bw[rc >> 5];
                               return (int)b.y + __popc(b.x & ((1u << (rc & 31)) - 1u)) - wb;
                           },
                           [&](int) {});
            wsync();
            if ((SPG_TILE_DIAG & 8) == 0) {   // (diag 8, timing only: no output)
                // values: the window's slots are its entries in C order
                T* __restrict__ xw = Cx + obase + wb;
                auto vals = [&](auto one) {   // 4 rows of 64 slots per round, reads first
                    for (int p0 = 0; p0 < wn; p0 += 4 * WAVE) {
                        T v[4];
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = S.acc[min(p0 + e * WAVE + l, SP_CAP + SP_DUMMY - 1)];
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const int p = p0 + e * WAVE + l;
                            if (p < wn) st_c(xw + p, decltype(one)::value ? v[e] : mul_rn(alpha, v[e]));
                        }
                    }
                };
                if (one) vals(std::true_type{});
                else vals(std::false_type{});
                wsync();
                // columns: each window lane lists its words' set bits at their ranks
                uint32_t* __restrict__ cl = reinterpret_cast<uint32_t*>(S.acc);
                if (l >= L0 && l < L1) {
                    int pos = p0 - wb;
#pragma unroll
                    for (int q = 0; q < SP_WPL; ++q) {
                        uint32_t w = wd[q];
                        const int cb = lo + 32 * (w0 + q);
                        while (w != 0u) {
                            cl[pos++] = (uint32_t)(cb + __builtin_ctz(w));
                            w &= w - 1u;
                        }
                    }
                }
                wsync();
                int32_t* __restrict__ cw = Cj + obase + wb;
                for (int p0 = 0; p0 < wn; p0 += 4 * WAVE) {
                    uint32_t v[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = cl[min(p0 + e * WAVE + l, SP_CAP - 1)];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int p = p0 + e * WAVE + l;
                        if (p < wn) st_c(cw + p, (int32_t)v[e]);
                    }
                }
            }
            L0 = L1;
        }
    }
}

// ---------------------------------------------------------------------------------------
// Symbolic pass over long B segments (a symbolic tile's expected segment >= SEG_MIN entries:
// config 4's whole rows of 328 columns, config 5's 65-column quarters).  The bitmap OR is
// order-free, so there is no lane -> product map: four A entries per instruction, one per
// 16-lane group, each group walking its entry's B segment 128 columns (one 16-byte load of
// eight 2-byte columns per lane, k_bj16) at a time, four entries per group in flight.  (Round 4: 16-byte
// loads -- a wave load costs the same per instruction whether it moves 4 or 16 bytes per lane,
// abtest/gather_probe -- instead of 4-byte ones: a quarter of the load instructions.)
// Writes each numeric tile's entry count (and, for sparse numeric tiles, its bitmap), as
// k_tile_sym.  (Measured on config 4: 4.05 ms against 7.05 ms for k_tile_sym's flattened
// walk over 16384-column tiles and 7.0 ms for a one-entry-per-instruction cursor walk.)
constexpr int SEG_WPB = 2;
#ifndef SPG_SYM_NQ
#define SPG_SYM_NQ 4   // (A/B: quads of A entries per round of k_tile_sym_seg)
#endif
// SPG_SYM_PF (round 6): the first SPG_SYM_PF steps of a k_tile_sym_seg round load together, with
// the next round's extents loaded under them (config 4 symbolic 2.74 -> 2.51 ms; 0: round 5's loop)
#ifndef SPG_SYM_PF
#define SPG_SYM_PF 3
#endif
// `ncols` > 0 (plans whose C rows are expected to be full, SPG_SYM_FULL in spgemm.hip): every 64
// A entries the wave counts its bitmap, and a task whose columns [lo, min(lo + width, ncols))
// are all set stops walking -- later products cannot add a column (config 3 at density 0.1:
// C rows 100 % dense, ~90 of 819 A entries fill a row).
template <typename IP>
__global__ __launch_bounds__(SEG_WPB * WAVE) void k_tile_sym_seg(
    int64_t row0, int64_t nrows, int tws, int G, int twss, const IP* __restrict__ Ap,
    const int32_t* __restrict__ Aj, const IP* __restrict__ Bp, const uint16_t* __restrict__ Bj16,
    const uint32_t* __restrict__ sidx, uint32_t* __restrict__ bitmap, int64_t* __restrict__ item_cnt,
    int64_t ncols) {
    constexpr int NQ = SPG_SYM_NQ;   // quads of A entries per round: 16 entries, 4 loads in flight per lane
    __shared__ __attribute__((aligned(16))) uint32_t bits_all[SEG_WPB][SYM_NWMAX];
    const int l = lane_id();
    const int sub = l & 15, grp = l >> 4;
    const int wv = uniform((int)(threadIdx.x >> 6));
    uint32_t* bits = bits_all[wv];
    const int nw = (1 << tws) >> 5;
    const int R = 1 << (twss - tws);
    const int Gs = (G + R - 1) / R;
    const uint32_t tasks = (uint32_t)(nrows * Gs);
    const uint32_t stride = gridDim.x * SEG_WPB;
    for (uint32_t task = xcd_block(gridDim.x) * SEG_WPB + wv; task < tasks; task += stride) {
        const int64_t row = row0 + (int64_t)(task / (uint32_t)Gs);
        const int gs = (int)(task % (uint32_t)Gs);
        const int t0 = gs * R, t1 = min(G, t0 + R);
        const int lo16 = (t0 << tws) & 0xffff;   // the tile's start inside its 65536-column block
        const int nws = (t1 - t0) * nw;
        const int64_t a0 = Ap[row];
        const int nA = (int)(Ap[row + 1] - a0);
        if (nA <= 0) {
            for (int t = t0 + l; t < t1; t += WAVE) item_cnt[(row - row0) * G + t] = 0;
            continue;
        }
        wsync();
        for (int w = l; w < nws; w += WAVE) bits[w] = 0u;
        wsync();
        // NQ quads of entries (4 per quad, one per 16-lane group) per round; the next round's
        // segment extents (A column -> B row start -> symbolic-tile start) are loaded while
        // this round's columns are in flight
        auto extents = [&](int b, int (&cnt)[NQ], int64_t (&beg)[NQ]) {
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                cnt[q] = 0;
                beg[q] = 0;
                const int e = b + 4 * q + grp;
                if (e < nA) {
                    const int32_t k = Aj[a0 + e];
                    const IP rb = Bp[k];
                    if (Gs == 1) {
                        cnt[q] = (int)(Bp[k + 1] - rb);
                        beg[q] = (int64_t)rb;
                    } else {
                        const uint32_t* sk = sidx + (int64_t)k * (Gs + 1);
                        const uint32_t s0 = sk[gs];
                        cnt[q] = (int)(sk[gs + 1] - s0);
                        beg[q] = (int64_t)rb + s0;
                    }
                }
            }
        };
        int cnt[NQ];
        int64_t beg[NQ];
        extents(0, cnt, beg);
        // the task's valid columns (the last tile of a row may pass the matrix's last column)
        const int full = ncols > 0 ? (int)min((int64_t)nws * 32, ncols - ((int64_t)t0 << tws)) : 0;
        // one round: NQ quads of A entries; eight 16-bit columns per lane per 16-byte load, each
        // segment from its 8-aligned start (span = cnt + (beg & 7) elements; an element before
        // beg or past the segment is skipped; the region is padded, so the last load stays
        // inside it).  A 16-lane group covers 128 columns per step; the longest span of the
        // round sets the steps.
        int odd[NQ], span[NQ];
        const uint4* __restrict__ w0[NQ];
        auto or_step = [&](int e, const uint4 (&w)[NQ]) {
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int x = e + 8 * sub;
                const uint32_t ww[4] = {w[q].x, w[q].y, w[q].z, w[q].w};
#pragma unroll
                for (int h = 0; h < 8; ++h) {
                    const int xh = x + h;
                    if (xh >= odd[q] && xh < span[q])
                        set_bit(bits, (int)((ww[h >> 1] >> (16 * (h & 1))) & 0xffffu) - lo16);
                }
            }
        };
        // (the loop is specialised for whole-row symbolic tiles, Gs == 1, so no uniform branch on
        // it sits between a load and its use)
        auto rounds = [&](auto gs1) {
            IP xr0[NQ], xr1[NQ];       // (SPG_SYM_PF: the next round's B row starts / ends,
            uint32_t xs0[NQ], xs1[NQ];  // or its symbolic-tile bounds, as loaded)
            bool pend = false;
            for (int b = 0; b < nA; b += 4 * NQ) {
                if (full > 0 && b > 0 && (b & (WAVE - 1)) == 0) {   // every 64 entries: full yet?
                    wsync();
                    int c = 0;
                    for (int w = l; w < nws; w += WAVE) c += __popc(bits[w]);
                    c = wave_incl_sum_dpp(c);
                    if (readlane_i(c, WAVE - 1) >= full) break;
                }
                if (SPG_SYM_PF > 0 && pend) {   // this round's extents from the raw words loaded last round
#pragma unroll
                    for (int q = 0; q < NQ; ++q) {
                        const bool ok = b + 4 * q + grp < nA;
                        if constexpr (decltype(gs1)::value) {
                            cnt[q] = ok ? (int)(xr1[q] - xr0[q]) : 0;
                            beg[q] = ok ? (int64_t)xr0[q] : 0;
                        } else {
                            cnt[q] = ok ? (int)(xs1[q] - xs0[q]) : 0;
                            beg[q] = ok ? (int64_t)xr0[q] + xs0[q] : 0;
                        }
                    }
                }
                int mx = 0;
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    odd[q] = (int)(beg[q] & 7);
                    span[q] = cnt[q] + odd[q];
                    w0[q] = reinterpret_cast<const uint4*>(Bj16 + (beg[q] - odd[q]));
                    mx = max(mx, span[q]);
                }
                mx = max(mx, __shfl_xor(mx, 16, WAVE));
                mx = max(mx, __shfl_xor(mx, 32, WAVE));
                mx = uniform(mx);
                int e0 = 0;
                if constexpr (SPG_SYM_PF > 0) {
                    // round 6: the next round's A columns first, then this round's first SPG_SYM_PF
                    // steps of column loads (unconditional: an index past the segment re-reads its
                    // last 16 bytes and is masked), then the next round's B extents (waiting only for
                    // the A columns: the column loads stay in flight), then the ORs: about one memory
                    // round trip per round instead of one per step plus a dependent chain per quad
                    int32_t kn[NQ];
#pragma unroll
                    for (int q = 0; q < NQ; ++q) kn[q] = Aj[a0 + min(b + 4 * NQ + 4 * q + grp, nA - 1)];
                    uint4 w[SPG_SYM_PF > 0 ? SPG_SYM_PF : 1][NQ];
#pragma unroll
                    for (int st = 0; st < SPG_SYM_PF; ++st)
#pragma unroll
                        for (int q = 0; q < NQ; ++q) {
                            const int last = max(span[q] - 1, 0) >> 3;
                            w[st][q] = w0[q][min((st * 128 + 8 * sub) >> 3, last)];
                        }
                    // (raw words only: they are combined at the next round's start, so nothing waits
                    // for them before the ORs)
#pragma unroll
                    for (int q = 0; q < NQ; ++q) {
                        xr0[q] = Bp[kn[q]];
                        if constexpr (decltype(gs1)::value) {
                            xr1[q] = Bp[kn[q] + 1];
                        } else {
                            const uint32_t* sk = sidx + (int64_t)kn[q] * (Gs + 1);
                            xs0[q] = sk[gs];
                            xs1[q] = sk[gs + 1];
                        }
                    }
                    pend = true;
#pragma unroll
                    for (int st = 0; st < SPG_SYM_PF; ++st)
                        if (st * 128 < mx) or_step(st * 128, w[st]);
                    e0 = SPG_SYM_PF * 128;
                }
                for (int e = e0; e < mx; e += 128) {
                    uint4 w[NQ];
#pragma unroll
                    for (int q = 0; q < NQ; ++q) {
                        const int x = e + 8 * sub;
                        w[q] = x < span[q] ? w0[q][x >> 3] : make_uint4(0u, 0u, 0u, 0u);
                    }
                    if (SPG_SYM_PF == 0 && e == 0) extents(b + 4 * NQ, cnt, beg);   // (next round; span/odd/w0 are kept)
                    or_step(e, w);
                }
                if (SPG_SYM_PF == 0 && mx == 0) extents(b + 4 * NQ, cnt, beg);
            }
        };
        if (Gs == 1) rounds(std::true_type{});
        else rounds(std::false_type{});
        wsync();
        if (bitmap) {
            uint32_t* __restrict__ out = bitmap + ((row - row0) * G + t0) * (int64_t)nw;
            for (int w = l; w < nws; w += WAVE) out[w] = bits[w];
        }
        for (int t = l; t < t1 - t0; t += WAVE) {
            int c = 0;
            for (int q = 0; q < nw; ++q) c += __popc(bits[t * nw + ((q + t) & (nw - 1))]);
            item_cnt[(row - row0) * G + t0 + t] = c;
        }
    }
}

}  // namespace spg
