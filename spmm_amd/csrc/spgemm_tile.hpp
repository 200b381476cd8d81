// spgemm_tile.hpp -- the wide-row path: work items are (output row, column tile) pairs.
//
// Rows whose A row is long or whose C row is wide (BASELINE configs 3 at density >= 1e-2,
// 4 and 5) are cut into column tiles of TW columns, so one row's work spreads over many
// waves.  A B column-tile index (for every B row k and tile g, the offset of the row's first
// entry with column >= g*TW) gives every item its B segments without searching.  Inside an
// item the products are enumerated in flattened (jj, kk) order exactly as in the short-row
// kernel (batches of 64 A entries, marker + DPP max-scan lane map, bitmap + popcount
// positions, lowest-lane-first owner rounds), so the result is bit-identical to scipy.
// Items whose structure exceeds CAP entries are processed in column windows of whole
// bitmap words, re-reading their products.
#pragma once

#include "spgemm_kernels.hpp"

namespace spg {

constexpr int TILE_WPB = 2;           // waves per block
constexpr int TILE_CAP = 1024;        // entries per window
constexpr int TILE_NWMAX = 128;       // bitmap words per tile: TW <= 4096 columns
constexpr int TILE_MK = 1024;         // marker bytes: 16 chunks of 64 products per group

template <typename T, typename IP, bool VALS> struct TileLds {
    uint32_t bits[TILE_NWMAX];
    uint16_t wpre[TILE_NWMAX];
    T acc[VALS ? TILE_CAP : 1];
    uint32_t tag[VALS ? TILE_CAP : 1];
    T ja[WAVE];
    IP jb0[WAVE];
    uint32_t joff[WAVE];
    int8_t mk[TILE_MK];
};

// Numeric tile pass LDS: the bitmap word and its popcount prefix side by side (one 8-byte
// read per product), the A-entry table as one 16-byte entry per lane.
template <typename T, typename IP> struct __attribute__((aligned(16))) TileEnt {
    IP jb0;          // first B index of the entry's segment
    uint32_t joff;   // flattened offset of the segment's first product
    T ja;            // the A value
};
template <typename T, typename IP> struct NumLds {
    uint2 bw[TILE_NWMAX];   // (bitmap word, popcount prefix)
    T acc[TILE_CAP];
    uint32_t tag[TILE_CAP];
    TileEnt<T, IP> ent[WAVE];
    int8_t mk[TILE_MK];
};

// ---------------------------------------------------------------------------------------
// B column-tile index: tidx[k*G + g] = (start, end) of B row k's entries with columns in
// tile g, as offsets inside the row (one 8-byte load per segment).  start_g = first entry
// with column >= g*TW.  One wave per B row; entries are sorted, so each boundary is
// written by the entry where the tile id steps.
template <typename IP>
__global__ __launch_bounds__(256) void k_tile_index(int64_t rows, const IP* __restrict__ Bp,
                                                    const int32_t* __restrict__ Bj, int tws, int G,
                                                    uint2* __restrict__ tidx) {
    const int l = lane_id();
    const int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (k >= rows) return;
    const IP r0 = Bp[k];
    const int len = (int)(Bp[k + 1] - r0);
    uint32_t* out = reinterpret_cast<uint32_t*>(tidx + k * (int64_t)G);
    auto put = [&](int g, uint32_t v) {   // boundary g: start of tile g, end of tile g-1
        if (g < G) out[2 * g] = v;
        if (g > 0) out[2 * g - 1] = v;
    };
    for (int e0 = 0; e0 < len; e0 += WAVE) {
        const int e = e0 + l;
        const int t = e < len ? Bj[r0 + e] >> tws : G;          // tile of this entry
        int tp = __shfl_up(t, 1, WAVE);                         // tile of the previous entry
        if (l == 0) tp = e0 == 0 ? -1 : (Bj[r0 + e0 - 1] >> tws);
        if (e < len)
            for (int g = tp + 1; g <= t; ++g) put(g, (uint32_t)e);
    }
    // boundaries after the last entry (and all of an empty row) are at len
    const int tl = len > 0 ? Bj[r0 + len - 1] >> tws : -1;
    for (int g = tl + 1 + l; g <= G; g += WAVE) put(g, (uint32_t)len);
}

// B packed as (column, value) records for the numeric tile pass: one load brings both.
template <typename T> struct BRec { int32_t c; int32_t pad; T v; };   // complex: 16 / 24 B
template <> struct __attribute__((aligned(16))) BRec<double> { int32_t c; int32_t pad; double v; };
template <> struct __attribute__((aligned(8))) BRec<float> { int32_t c; float v; };

// One load per record: 16 bytes (f64) or 8 bytes (f32).
template <typename T, typename IP>
__device__ __forceinline__ void load_rec(const BRec<T>* __restrict__ rec, IP i, int& c, T& v) {
    if constexpr (!std::is_same<T, double>::value && !std::is_same<T, float>::value) {
        c = rec[i].c;
        v = rec[i].v;
    } else if constexpr (sizeof(T) == 8) {
        const uint4 q = reinterpret_cast<const uint4*>(rec)[i];
        c = (int)q.x;
        v = __hiloint2double((int)q.w, (int)q.z);
    } else {
        const uint2 q = reinterpret_cast<const uint2*>(rec)[i];
        c = (int)q.x;
        v = __uint_as_float(q.y);
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_pack_b(int64_t nnz, const int32_t* __restrict__ Bj,
                                                const T* __restrict__ Bx, BRec<T>* __restrict__ rec) {
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nnz; e += (int64_t)gridDim.x * 256) {
        BRec<T> r;
        r.c = Bj[e];
        if constexpr (!std::is_same<T, float>::value) r.pad = 0;
        r.v = Bx[e];
        rec[e] = r;
    }
}

// Blocks are dispatched round-robin over the 8 XCDs.  Logical block ids that keep
// consecutive ids on one XCD make the tiles of one row share that XCD's L2 (they read the
// same B rows).  `nb` (the grid) is a multiple of 8.
__device__ __forceinline__ uint32_t xcd_block(uint32_t nb) {
    const uint32_t b = blockIdx.x;
    return (b & 7u) * (nb >> 3) + (b >> 3);
}

constexpr int SYM_NWMAX = 2048;   // symbolic bitmap words: 65536 columns

template <typename IP> struct SymLds {
    uint32_t bits[SYM_NWMAX];
    IP jb0[WAVE];
    uint32_t joff[WAVE];
    int8_t mk[TILE_MK];
};

// Lane -> A-entry map for a group of up to 16 chunks (1024 products) starting at gbase.
template <typename L>
__device__ __forceinline__ void group_markers(L& S, int l, int cnt, int off, int gbase) {
    wsync();
    reinterpret_cast<uint4*>(S.mk)[l] = make_uint4(~0u, ~0u, ~0u, ~0u);
    wsync();
    if (cnt > 0 && off >= gbase && off < gbase + TILE_MK) S.mk[off - gbase] = (int8_t)l;
    wsync();
}

// Chunks of one group (<= 16 x 64 products) U at a time: map lanes to A entries for U
// chunks, issue all their B loads, then hand each chunk to `fn(col, bval, aval)` in order
// (lanes past the group's products get col = -1).
template <int U, bool VALS, typename T, typename IP, typename L, typename F>
__device__ __forceinline__ void walk_group(L& S, int l, int gb, int Pb, int& carry,
                                           const int32_t* __restrict__ Bj,
                                           const T* __restrict__ Bx, F&& fn,
                                           const BRec<T>* __restrict__ rec = nullptr) {
    const int nchg = min(TILE_MK, Pb - gb);
    for (int c0 = 0; c0 < nchg; c0 += U * WAVE) {
        IP idx[U];
        T av[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            idx[u] = (IP)-1;
            av[u] = (T)0;
            const int cc = c0 + u * WAVE;
            if (cc < nchg) {
                const int src = max(wave_incl_max_dpp((int)S.mk[cc + l]), carry);
                carry = readlane_i(src, WAVE - 1);
                const int t = gb + cc + l;
                if (t < Pb) {
                    idx[u] = S.jb0[src] + (IP)(t - (int)S.joff[src]);
                    if constexpr (VALS) av[u] = S.ja[src];
                }
            }
        }
        int col[U];
        T bv[U];
        if (VALS && rec) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                col[u] = -1;
                bv[u] = (T)0;
                if (idx[u] >= 0) {
                    const BRec<T> r = rec[idx[u]];
                    col[u] = r.c;
                    bv[u] = r.v;
                }
            }
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                col[u] = idx[u] >= 0 ? Bj[idx[u]] : -1;
                bv[u] = (VALS && idx[u] >= 0) ? Bx[idx[u]] : (T)0;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (c0 + u * WAVE < nchg) fn(col[u], bv[u], av[u]);
    }
}

// Symbolic pass of the tile path over wide symbolic tiles: R = 2^(twss - tws) numeric
// tiles at once (up to 65536 columns, the whole row for N <= 65536), so B rows are read in
// long coalesced segments.  Writes each numeric tile's bitmap (contiguous per row) and its
// entry count.
template <typename IP>
__global__ __launch_bounds__(TILE_WPB * WAVE) void k_tile_sym(
    int64_t row0, int64_t nrows, int tws, int G, int twss, const IP* __restrict__ Ap,
    const int32_t* __restrict__ Aj, const IP* __restrict__ Bp, const int32_t* __restrict__ Bj,
    const uint2* __restrict__ tidx, uint32_t* __restrict__ bitmap, int64_t* __restrict__ item_cnt) {
    __shared__ __attribute__((aligned(16))) SymLds<IP> lds[TILE_WPB];
    const int l = lane_id();
    const int wv = uniform((int)(threadIdx.x >> 6));
    SymLds<IP>& S = lds[wv];
    const int nw = (1 << tws) >> 5;           // words of a numeric tile
    const int R = 1 << (twss - tws);          // numeric tiles per symbolic tile
    const int Gs = (G + R - 1) / R;           // symbolic tiles per row
    const uint32_t tasks = (uint32_t)(nrows * Gs);
    const uint32_t stride = gridDim.x * TILE_WPB;
    for (uint32_t task = xcd_block(gridDim.x) * TILE_WPB + wv; task < tasks; task += stride) {
        const int64_t row = row0 + (int64_t)(task / (uint32_t)Gs);
        const int gs = (int)(task % (uint32_t)Gs);
        const int t0 = gs * R, t1 = min(G, t0 + R);
        const int lo = t0 << tws;
        const int nws = (t1 - t0) * nw;
        const int64_t a0 = Ap[row];
        const int nA = (int)(Ap[row + 1] - a0);
        if (nA <= 0) {
            for (int t = t0 + l; t < t1; t += WAVE) item_cnt[row * G + t] = 0;
            continue;
        }
        wsync();
        for (int w = l; w < nws; w += WAVE) S.bits[w] = 0u;
        for (int b = 0; b < nA; b += WAVE) {
            int cnt = 0;
            IP beg = 0;
            if (b + l < nA) {
                const int32_t k = Aj[a0 + b + l];
                const IP rb = Bp[k];
                if (Gs == 1) {
                    cnt = (int)(Bp[k + 1] - rb);
                    beg = rb;
                } else {
                    const uint2* tk = tidx + (int64_t)k * G;
                    const uint32_t s0 = tk[t0].x;
                    cnt = (int)(tk[t1 - 1].y - s0);
                    beg = rb + (IP)s0;
                }
            }
            const int incl = wave_incl_sum_dpp(cnt);
            const int off = incl - cnt;
            const int Pb = readlane_i(incl, WAVE - 1);
            wsync();
            S.jb0[l] = beg;
            S.joff[l] = (uint32_t)off;
            wsync();
            int carry = -1;
            for (int gb = 0; gb < Pb; gb += TILE_MK) {
                group_markers(S, l, cnt, off, gb);
                walk_group<8, false, float, IP>(S, l, gb, Pb, carry, Bj, (const float*)nullptr,
                                               [&](int c, float, float) {
                                                   if (c >= 0) set_bit(S.bits, c - lo);
                                               });
            }
        }
        wsync();
        uint32_t* __restrict__ out = bitmap + (row * G + t0) * (int64_t)nw;
        for (int w = l; w < nws; w += WAVE) out[w] = S.bits[w];
        // entry count of each numeric tile: lane t sums tile t's words (rotated start: no
        // two lanes read one bank together)
        for (int t = l; t < t1 - t0; t += WAVE) {
            int c = 0;
            for (int j = 0; j < nw; ++j) c += __popc(S.bits[t * nw + ((j + t) & (nw - 1))]);
            item_cnt[row * G + t0 + t] = c;
        }
    }
}

// Numeric pass of the tile path: one wave per item (row, numeric tile).  Reads the item's
// bitmap from the symbolic pass, enumerates its products in flattened (jj, kk) order --
// one 8-byte index load per A entry, one record load per product from the packed B --
// and accumulates lowest-lane-first per output position; items with more than CAP entries
// go in column windows (products re-read per window).
template <typename T, typename IP>
__global__ __launch_bounds__(TILE_WPB * WAVE) void k_tile(
    int64_t row0, int64_t nrows, int tws, int G, const IP* __restrict__ Ap,
    const int32_t* __restrict__ Aj, const T* __restrict__ Ax, const IP* __restrict__ Bp,
    const BRec<T>* __restrict__ brec, const uint2* __restrict__ tidx,
    const uint32_t* __restrict__ bitmap, const int64_t* __restrict__ item_off,
    int32_t* __restrict__ Cj, T* __restrict__ Cx, T alpha) {
    constexpr int U = sizeof(T) > 8 ? 4 : 8;   // chunks in flight (complex128: half)
    __shared__ __attribute__((aligned(16))) NumLds<T, IP> lds[TILE_WPB];
    const int l = lane_id();
    const int wv = uniform((int)(threadIdx.x >> 6));
    NumLds<T, IP>& S = lds[wv];
    const int TW = 1 << tws;
    const int nw = TW >> 5;                    // bitmap words of a tile
    const int wpl = (nw + WAVE - 1) / WAVE;    // words per lane (<= 2)
    const uint32_t items = (uint32_t)(nrows * G);   // host keeps rows*G < 2^31
    for (uint32_t it = xcd_block(gridDim.x) * TILE_WPB + wv; it < items; it += gridDim.x * TILE_WPB) {
        const int64_t row = row0 + (int64_t)(it / (uint32_t)G);
        const int g = (int)(it % (uint32_t)G);
        const int64_t item = row * G + g;
        const int lo = g * TW;
        const int64_t a0 = Ap[row];
        const int nA = (int)(Ap[row + 1] - a0);
        if (nA <= 0) continue;
        const uint32_t* __restrict__ ibits = bitmap + item * nw;
        // the symbolic bitmap and its popcount prefix (lane owns wpl words)
        const int w0 = min(nw, l * wpl), w1 = min(nw, w0 + wpl);
        uint32_t wd[2] = {0u, 0u};
        int mine = 0;
#pragma unroll
        for (int q = 0; q < 2; ++q)
            if (w0 + q < w1) {
                wd[q] = ibits[w0 + q];
                mine += __popc(wd[q]);
            }
        const int pincl = wave_incl_sum_dpp(mine);
        const int nnz = readlane_i(pincl, WAVE - 1);
        if (nnz == 0) continue;
        const int p0 = pincl - mine;
        wsync();
        {
            int run = p0;
#pragma unroll
            for (int q = 0; q < 2; ++q)
                if (w0 + q < w1) {
                    S.bw[w0 + q] = make_uint2(wd[q], (uint32_t)run);
                    run += __popc(wd[q]);
                }
        }
        wsync();
        const int64_t obase = item_off[item];
        // The first NB batches of A entries (rows of <= NB*64 entries: all of them): every
        // lane's A entry, value, tile segment and B row start, loaded at once up front (two
        // dependent load levels per item instead of two per batch).
        constexpr int NB = sizeof(T) > 8 ? 4 : 8;
        int32_t kq[NB];
        T aq[NB];
        uint2 sq[NB];
        IP bq[NB];
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            kq[q] = -1;
            aq[q] = (T)0;
            if (q * WAVE < nA && q * WAVE + l < nA) {
                kq[q] = Aj[a0 + q * WAVE + l];
                aq[q] = Ax[a0 + q * WAVE + l];
            }
        }
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            sq[q] = make_uint2(0u, 0u);
            bq[q] = 0;
            if (kq[q] >= 0) {
                sq[q] = tidx[(int64_t)kq[q] * G + g];
                bq[q] = Bp[kq[q]];
            }
        }
        // lane info of one batch of A entries: (first B index, count) of its tile segment
        auto batch = [&](int b, int& cnt, int& off, int& Pb) {
            cnt = 0;
            IP beg = 0;
            T av = (T)0;
            if (b < NB * WAVE) {
#pragma unroll
                for (int q = 0; q < NB; ++q)
                    if (q == (b >> 6)) {
                        cnt = (int)(sq[q].y - sq[q].x);
                        beg = bq[q] + (IP)sq[q].x;
                        av = aq[q];
                    }
            } else if (b + l < nA) {
                const int32_t k = Aj[a0 + b + l];
                const uint2 se = tidx[(int64_t)k * G + g];
                cnt = (int)(se.y - se.x);
                beg = Bp[k] + (IP)se.x;
                av = Ax[a0 + b + l];
            }
            const int incl = wave_incl_sum_dpp(cnt);
            off = incl - cnt;
            Pb = readlane_i(incl, WAVE - 1);
            wsync();
            S.ent[l] = TileEnt<T, IP>{beg, (uint32_t)off, av};
            wsync();
        };
        for (int L0 = 0; L0 < WAVE;) {
            int L1 = WAVE, wb = 0, wn = nnz;
            if (nnz > TILE_CAP) {
                wb = readlane_i(p0, L0);
                L1 = (int)__popcll(__ballot(pincl <= wb + TILE_CAP));
                if (L1 <= L0) L1 = L0 + 1;
                wn = (L1 < WAVE ? readlane_i(p0, L1) : nnz) - wb;
            }
            const int clo = lo + 32 * wpl * L0, chi = lo + 32 * wpl * L1;
            for (int p = l; p < wn; p += WAVE) {
                S.acc[p] = (T)0;
                S.tag[p] = 0xffffffffu;
            }
            wsync();
            uint32_t seq = 0x7fffffu;   // 23 bits: key = seq | chunk (3 bits) | lane (6 bits)
            for (int b = 0; b < nA; b += WAVE) {
                int cnt, off, Pb;
                batch(b, cnt, off, Pb);
                int carry = -1;
                for (int gb = 0; gb < Pb; gb += TILE_MK) {
                    group_markers(S, l, cnt, off, gb);
                    const int nchg = min(TILE_MK, Pb - gb);
                    for (int c0 = 0; c0 < nchg; c0 += U * WAVE) {
                        // lane -> A entry of U chunks at once; chunks past the group read the
                        // -1 markers, so `carry` passes through them unchanged.  Indices of
                        // lanes past the group are clamped to 0 and their results dropped.
                        IP idx[U];
                        T av[U];
                        bool val[U];
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            const int cc = c0 + u * WAVE;
                            const int src = max(wave_incl_max_dpp((int)S.mk[cc + l]), carry);
                            carry = readlane_i(src, WAVE - 1);
                            const int t = gb + cc + l;
                            val[u] = t < Pb;
                            const TileEnt<T, IP> e = S.ent[max(src, 0)];
                            idx[u] = val[u] ? e.jb0 + (IP)(t - (int)e.joff) : (IP)0;
                            av[u] = e.ja;
                        }
                        int qc[U];
                        T qv[U];
#pragma unroll
                        for (int u = 0; u < U; ++u) load_rec(brec, idx[u], qc[u], qv[u]);
                        // positions and products of all U chunks, then one joint owner
                        // round for the U*64 products: key (seq, chunk, lane) orders them by
                        // flattened index, so the lowest pending product of every position
                        // adds first; a lane's U atomics are independent and pipeline
                        int pos[U];
                        T pv[U];
                        uint32_t pend = 0u;
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            const int c = (val[u] && c0 + u * WAVE < nchg) ? qc[u] : -1;
                            pos[u] = 0;
                            if (c >= clo && c < chi) {
                                const int rc = c - lo;
                                const uint2 bw = S.bw[rc >> 5];
                                pos[u] = (int)bw.y + __popc(bw.x & ((1u << (rc & 31)) - 1u)) - wb;
                                pend |= 1u << u;
                            }
                            pv[u] = mul_rn(av[u], qv[u]);
                        }
                        while (__ballot(pend != 0u)) {
                            const uint32_t kb = (seq << 9) | (uint32_t)l;
#pragma unroll
                            for (int u = 0; u < U; ++u)
                                if (pend & (1u << u)) atomicMin(&S.tag[pos[u]], kb | ((uint32_t)u << 6));
#pragma unroll
                            for (int u = 0; u < U; ++u)
                                if ((pend & (1u << u)) &&
                                    __hip_atomic_load(&S.tag[pos[u]], __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_WAVEFRONT) == (kb | ((uint32_t)u << 6))) {
                                    S.acc[pos[u]] = add_rn(S.acc[pos[u]], pv[u]);
                                    pend &= ~(1u << u);
                                }
                            --seq;
                        }
                        if (seq < 4096u) {   // re-arm the tag space (very long items only)
                            wsync();
                            for (int p = l; p < wn; p += WAVE) S.tag[p] = 0xffffffffu;
                            seq = 0x7fffffu;
                            wsync();
                        }
                    }
                }
            }
            wsync();
            // column list of this window from the bitmap (lane-owned words)
            if (l >= L0 && l < L1) {
                int p = p0 - wb;
                for (int w = w0; w < w1; ++w) {
                    uint32_t x = S.bw[w].x;
                    while (x) {
                        S.tag[p++] = (uint32_t)(lo + 32 * w + __builtin_ctz(x));
                        x &= x - 1u;
                    }
                }
            }
            wsync();
            int32_t* __restrict__ crow = Cj + obase + wb;
            T* __restrict__ xrow = Cx + obase + wb;
            for (int p = l; p < wn; p += WAVE) {
                crow[p] = (int32_t)S.tag[p];
                const T val = S.acc[p];
                xrow[p] = (alpha == (T)1) ? val : mul_rn(alpha, val);
            }
            wsync();
            L0 = L1;
        }
    }
}

// C's row pointer from the per-item offsets: Cp[i] = item_off[i*G]; overflow flag when the
// total does not fit OUT.  Rows [row0, row0 + nrows) plus the final entry.
template <typename OUT>
__global__ __launch_bounds__(256) void k_items_to_rowptr(int64_t rows, int G,
                                                         const int64_t* __restrict__ item_off,
                                                         OUT* __restrict__ Cp) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i <= rows) Cp[i] = (OUT)item_off[i * G];
}

}  // namespace spg
