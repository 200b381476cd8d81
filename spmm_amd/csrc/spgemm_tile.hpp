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
// waves per block of the numeric kernel: sparse tiles (14 KB of LDS per wave) fit 11
// one-wave blocks per CU where 2-wave blocks fit 10; dense tiles (13 KB) fit 12 either way
template <bool DENSE> constexpr int tile_num_wpb() { return DENSE ? 2 : 1; }
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
    uint8_t mk[TILE_MK];
};

// Numeric tile pass LDS: the bitmap word and its popcount prefix side by side (one 8-byte
// read per product; sparse tiles only), the A-entry table as one 8-byte entry per lane (the
// A values stay in registers and reach the product lanes by a lane shuffle), the markers
// of 8 chunks.  Dense tiles thus take 13 KB per wave: 12 waves per CU (6 blocks of 2)
// instead of 10 at 15 KB.
constexpr int NUM_MK = 512;   // numeric marker bytes: 8 chunks of 64 products per group
template <typename IP> struct __attribute__((aligned(8))) TileSeg {
    IP jb0;          // first B index of the entry's segment
    uint32_t joff;   // flattened offset of the segment's first product
};
template <typename T, typename IP, bool DENSE> struct NumLds {
    uint2 bw[DENSE ? 1 : TILE_NWMAX];   // (bitmap word, popcount prefix)
    T acc[TILE_CAP];
    uint32_t tag[TILE_CAP];
    TileSeg<IP> ent[WAVE];
    uint8_t mk[NUM_MK];
};

// Numeric lane -> A-entry markers for a group of up to 8 chunks (512 products) starting at
// gbase, transposed as in group_markers: product t's marker at byte 8 * (t % 64) + t / 64,
// so each lane reads all 8 of its chunks' markers with one 8-byte LDS load.
template <typename L>
__device__ __forceinline__ void num_group_markers(L& S, int l, int cnt, int off, int gbase) {
    wsync();
    reinterpret_cast<uint2*>(S.mk)[l] = make_uint2(0u, 0u);
    wsync();
    if (cnt > 0 && off >= gbase && off < gbase + NUM_MK) {
        const int t = off - gbase;
        S.mk[((t & (WAVE - 1)) << 3) | (t >> 6)] = (uint8_t)(l + 1);
    }
    wsync();
}

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

// Tile-major B records: the entry's value followed by its column inside its tile (32 bits),
// packed without padding -- 8 bytes (f32), 12 bytes (f64, complex64), 20 bytes
// (complex128) -- so one dwordx2 / dwordx3 load brings both, and the slice of a tile the
// XCD keeps in L2 is as small as the values allow.  The value comes first so that an f64
// lands in the even-aligned register pair of the dwordx3 (no moves before the multiply).
// Offsets are 32-bit byte offsets from the (scalar) base: the host keeps the record array
// under 4 GiB on the tile path.
template <typename T> constexpr int rec_words() { return 1 + (int)(sizeof(T) / 4); }
// SPG_REC10 (round 4, default): fp64 records of 10 bytes -- the value, then the column inside the
// tile as u16 (tiles
// are at most 8192 columns wide, sentinel columns below 65536) -- packed without padding, so a
// tile's slice is 5/6 of the 12-byte form (config 4's 2048-column slice 8.0 -> 6.7 MB against an
// XCD's 4 MB L2).  Record i starts at byte 10i, which is 0 or 2 modulo 4: one dwordx3 load from
// the dword below it holds the whole record, and two v_alignbit and a shift take it apart.
// Measured (A/B on one box): config 4 numeric 20.7 -> 19.8 ms, config 5 103.7 -> 98.7 ms.
#ifndef SPG_REC10
#define SPG_REC10 1
#endif
// SPG_REC6 (round 5, default): fp32 records of 6 bytes the same way -- the value, then the column
// inside the tile as u16 (fp32 tiles are at most 4096 columns wide) -- record i at byte 6i (0 or 2
// modulo 4): one dwordx2 from the dword below it, one v_alignbit.  8 -> 6 bytes per product of
// gather traffic for the fp32 tile kernels.
#ifndef SPG_REC6
#define SPG_REC6 1
#endif
template <typename T> constexpr int rec_bytes() {
    return (SPG_REC10 && std::is_same<T, double>::value) ? 10
           : (SPG_REC6 && std::is_same<T, float>::value) ? 6 : 4 * rec_words<T>();
}

#ifndef SPG_REC_NT
#define SPG_REC_NT 0   // (A/B: record gathers with the non-temporal policy, bypassing the CU's L1)
#endif
typedef unsigned int spg_u32x3 __attribute__((ext_vector_type(3)));
template <typename T, typename IP>
__device__ __forceinline__ void load_rec(const uint32_t* __restrict__ rec, IP i, int& lc, T& v) {
    constexpr int W = rec_words<T>();
    if constexpr (rec_bytes<T>() == 10) {   // fp64, 10-byte records
        const char* p = reinterpret_cast<const char*>(rec) + (uint64_t)((uint32_t)i * 10u);
        const uint32_t sh = (uint32_t)((uintptr_t)p & 2u) * 8u;     // 0 or 16 bits
        uint3 x;
        if constexpr (SPG_REC_NT) {
            const spg_u32x3 y = __builtin_nontemporal_load(reinterpret_cast<const spg_u32x3*>(p - ((uintptr_t)p & 2u)));
            x = make_uint3(y.x, y.y, y.z);
        } else {
            x = *reinterpret_cast<const uint3*>(p - ((uintptr_t)p & 2u));
        }
        const uint32_t lo = __builtin_amdgcn_alignbit(x.y, x.x, sh);
        const uint32_t hi = __builtin_amdgcn_alignbit(x.z, x.y, sh);
        v = __hiloint2double((int)hi, (int)lo);
        lc = (int)((x.z >> sh) & 0xffffu);
        return;
    } else if constexpr (rec_bytes<T>() == 6) {   // fp32, 6-byte records
        const char* p = reinterpret_cast<const char*>(rec) + (uint64_t)((uint32_t)i * 6u);
        const uint32_t sh = (uint32_t)((uintptr_t)p & 2u) * 8u;
        const uint2 x = *reinterpret_cast<const uint2*>(p - ((uintptr_t)p & 2u));
        v = __uint_as_float(__builtin_amdgcn_alignbit(x.y, x.x, sh));
        lc = (int)((x.y >> sh) & 0xffffu);
        return;
    }
    const uint32_t* __restrict__ q =
        reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(rec) + (uint64_t)((uint32_t)i * (uint32_t)(4 * W)));
    if constexpr (W == 2) {          // f32
        const uint2 x = *reinterpret_cast<const uint2*>(q);
        v = __uint_as_float(x.x);
        lc = (int)x.y;
    } else if constexpr (W == 3) {   // f64, complex64
        const uint3 x = *reinterpret_cast<const uint3*>(q);
        if constexpr (std::is_same<T, double>::value) {
            v = __hiloint2double((int)x.y, (int)x.x);
        } else {
            v.re = __uint_as_float(x.x);
            v.im = __uint_as_float(x.y);
        }
        lc = (int)x.z;
    } else {                          // complex128
        __builtin_memcpy(&v, q, sizeof(T));
        lc = (int)q[W - 1];
    }
}

// Record at BYTE offset `off` from the (uniform) base `rb`: the 32-bit offset reaches the load
// as its VGPR offset with the base in SGPRs (global_load ... v_off, s[base]), one VGPR per
// address instead of a 64-bit pair, no 64-bit address arithmetic per product.
template <typename T>
__device__ __forceinline__ void load_rec_at(const char* __restrict__ rb, uint32_t off, int& lc, T& v) {
    if constexpr (rec_bytes<T>() == 10) {
        const uint32_t sh = (off & 2u) * 8u;   // records start at 0 or 2 modulo 4
        uint3 x;
        if constexpr (SPG_REC_NT) {
            const spg_u32x3 y = __builtin_nontemporal_load(reinterpret_cast<const spg_u32x3*>(rb + (off & ~3u)));
            x = make_uint3(y.x, y.y, y.z);
        } else {
            x = *reinterpret_cast<const uint3*>(rb + (off & ~3u));
        }
        const uint32_t lo = __builtin_amdgcn_alignbit(x.y, x.x, sh);
        const uint32_t hi = __builtin_amdgcn_alignbit(x.z, x.y, sh);
        v = __hiloint2double((int)hi, (int)lo);
        lc = (int)((x.z >> sh) & 0xffffu);
    } else if constexpr (rec_bytes<T>() == 6) {
        const uint32_t sh = (off & 2u) * 8u;
        const uint2 x = *reinterpret_cast<const uint2*>(rb + (off & ~3u));
        v = __uint_as_float(__builtin_amdgcn_alignbit(x.y, x.x, sh));
        lc = (int)((x.y >> sh) & 0xffffu);
    } else {
        load_rec(reinterpret_cast<const uint32_t*>(rb + off), 0, lc, v);
    }
}

template <typename T>
__device__ __forceinline__ void store_rec(uint32_t* __restrict__ rec, int64_t i, int lc, T v) {
    if constexpr (rec_bytes<T>() == 6) {   // three 2-byte stores
        uint16_t* q = reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(rec) + i * 6);
        const uint32_t b = __float_as_uint(v);
        q[0] = (uint16_t)b;
        q[1] = (uint16_t)(b >> 16);
        q[2] = (uint16_t)lc;
        return;
    }
    if constexpr (rec_bytes<T>() == 10) {   // five 2-byte stores (a record is 2-byte aligned)
        uint16_t* q = reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(rec) + i * 10);
        uint64_t b;
        __builtin_memcpy(&b, &v, 8);
#pragma unroll
        for (int h = 0; h < 4; ++h) q[h] = (uint16_t)(b >> (16 * h));
        q[4] = (uint16_t)lc;
        return;
    }
    constexpr int W = rec_words<T>();
    uint32_t* q = rec + i * W;
    __builtin_memcpy(q, &v, sizeof(T));
    q[W - 1] = (uint32_t)lc;
}

// The column part / the value part of a record alone (spg_numeric_tiles: columns from B's
// structure first, values group by group as they arrive).
template <typename T>
__device__ __forceinline__ void store_rec_col(uint32_t* __restrict__ rec, int64_t i, int lc) {
    if constexpr (rec_bytes<T>() == 6) {
        reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(rec) + i * 6)[2] = (uint16_t)lc;
    } else if constexpr (rec_bytes<T>() == 10) {
        reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(rec) + i * 10)[4] = (uint16_t)lc;
    } else {
        rec[i * rec_words<T>() + rec_words<T>() - 1] = (uint32_t)lc;
    }
}
template <typename T>
__device__ __forceinline__ void store_rec_val(uint32_t* __restrict__ rec, int64_t i, T v) {
    if constexpr (rec_bytes<T>() == 6) {
        uint16_t* q = reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(rec) + i * 6);
        const uint32_t b = __float_as_uint(v);
        q[0] = (uint16_t)b;
        q[1] = (uint16_t)(b >> 16);
    } else if constexpr (rec_bytes<T>() == 10) {
        uint16_t* q = reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(rec) + i * 10);
        uint64_t b;
        __builtin_memcpy(&b, &v, 8);
#pragma unroll
        for (int h = 0; h < 4; ++h) q[h] = (uint16_t)(b >> (16 * h));
    } else {
        __builtin_memcpy(rec + i * rec_words<T>(), &v, sizeof(T));
    }
}

// Sentinel records after B's nnz records: the lean tile kernels point every product slot past
// the end of a batch at them instead of masking the slot (no compare / select per chunk).
// Regions 0, 1 and 3 (dense tiles of 1024 / 2048 / 4096 columns): columns 1024 / 2048 / 4096 + (i % 32),
// accumulator slots nobody reads; region 2 (sparse tiles, <= 8192 columns): columns
// 65472 + (i % 64), outside every window (and within the 10-byte records' u16).  Value 0.
constexpr int SENT_N = 512;        // records per region: a step never runs more than 512 slots past its batch
constexpr int SENT_REGIONS = 4;
constexpr int DN_DUMMY = 32;       // accumulator slots past a dense tile: the sentinel records add into them
// SPG_DN_WIDE_TWS: log2 of the widest fp64 dense tile (11: 2048 columns; 12: 4096, A/B builds)
#ifndef SPG_DN_WIDE_TWS
#define SPG_DN_WIDE_TWS 11
#endif
constexpr int DN_TW_MAX = 1 << SPG_DN_WIDE_TWS;   // widest dense tile (fp64: its accumulator's slots)
__device__ __forceinline__ int sentinel_col(int i) {
    const int r = i / SENT_N, x = i % SENT_N;
    return r == 0 ? 1024 + (x & (DN_DUMMY - 1)) : r == 1 ? 2048 + (x & (DN_DUMMY - 1))
                                                : r == 3 ? 4096 + (x & (DN_DUMMY - 1)) : 0xffc0 + (x & 63);
}
__host__ __device__ constexpr int sentinel_region(int dense_tw) {
    return dense_tw == 1024 ? 0 : dense_tw == 2048 ? 1 : dense_tw == 4096 ? 3 : 2;
}

// ---------------------------------------------------------------------------------------
// Tile-major B in record groups.  Tiles are taken RG = 1 << rgs at a time (a record group:
// RG adjacent column tiles); for every group, B's entries with columns in the group, row by
// row, and inside a row tile by tile -- i.e. the tile-major layout of tiles RG times as wide,
// whose every row segment is cut at the RG - 1 inner tile boundaries.  The group's segment
// table has K*RG + 1 words: word k*RG + t is the offset of row k's segment of tile t of the
// group, and its successor (word k*RG + t + 1) is that segment's end -- the next tile's start
// in the same row, or the next row's first segment; word K*RG is the group's end.  With
// RG = 1 this is the plain tile-major layout: tile g's table at g*(K+1), one word per row.
// A (row, tile) item finds each A entry's segment with two adjacent 4-byte loads; the RG
// tiles of one row read ONE contiguous run of records per B row (k_tile_sp's cooperative
// blocks walk it with one wave per tile, so a cache line carries the segments of several
// tiles instead of one).  Built once per plan from the row-major boundary index (k_tile_index
// over the group-padded tile count, a temporary):
//   k_bt_count   segment lengths into tptr and symbolic-tile starts into sidx
//   k_scan_lb    lengths -> offsets, in place
//   k_bt_pack    every B entry to its place (column, value record)
// Segment table of tile g (its words at stride RG from there).
__host__ __device__ __forceinline__ int64_t tile_table_off(int g, int64_t K, int rgs) {
    return (int64_t)(g >> rgs) * ((K << rgs) + 1) + (g & ((1 << rgs) - 1));
}
// Gp = the group-padded tile count (a multiple of RG); tiles g >= G (padding) get no entries.
__global__ __launch_bounds__(256) void k_bt_count(int64_t K, int Gp, int G, int R, const uint2* __restrict__ tidx,
                                                  int32_t* __restrict__ tptr, uint32_t* __restrict__ sidx, int rgs) {
    const int64_t n = K * Gp;
    const int Gs = (G + R - 1) / R;
    const int Gq = Gp >> rgs;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n + Gq; i += (int64_t)gridDim.x * 256) {
        if (i >= n) {   // the end slot of each group
            tptr[(i - n) * ((K << rgs) + 1) + (K << rgs)] = 0;
            continue;
        }
        const int64_t k = i / Gp;
        const int g = (int)(i - k * Gp);
        const uint2 se = tidx[i];
        tptr[tile_table_off(g, K, rgs) + (k << rgs)] = (int32_t)(se.y - se.x);
        if (g < G && g % R == 0) sidx[k * (Gs + 1) + g / R] = se.x;
        if (g == G - 1) sidx[k * (Gs + 1) + Gs] = se.y;
    }
}

// One wave per B row: an entry's rank inside its tile segment is its distance to the
// segment's first entry, found by a max-scan over the lanes where the tile id steps.
// (The grid's first SENT_REGIONS * SENT_N threads also write the sentinel records after the
// nnz(B) real ones.)
// MODE 0: whole records; 1: the column parts and the sentinels only (values come later,
// k_bt_fill); 2: the values alone, densely in record order into `tm` (spg_tile_values).
template <typename T, typename IP, int MODE = 0>
__global__ __launch_bounds__(256) void k_bt_pack(int64_t K, const IP* __restrict__ Bp, const int32_t* __restrict__ Bj,
                                                 const T* __restrict__ Bx, int tws,
                                                 const int32_t* __restrict__ tptr, uint32_t* __restrict__ rec,
                                                 int64_t nnzB, T* __restrict__ tm, int rgs) {
    const int l = lane_id();
    if (MODE != 2)
        for (int i = blockIdx.x * 256 + threadIdx.x; i < SENT_REGIONS * SENT_N; i += gridDim.x * 256)
            store_rec(rec, nnzB + i, sentinel_col(i), (T)0);
    const int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (k >= K) return;
    const IP r0 = Bp[k];
    const int len = (int)(Bp[k + 1] - r0);
    int carry = 0;   // first entry of the segment the previous chunk ended in
    for (int e0 = 0; e0 < len; e0 += WAVE) {
        const int e = e0 + l;
        const bool in = e < len;
        const int32_t c = in ? Bj[r0 + e] : 0;
        const int g = c >> tws;
        int gp = __shfl_up(g, 1, WAVE);
        if (l == 0) gp = e0 == 0 ? -1 : (Bj[r0 + e0 - 1] >> tws);
        const int s0 = max(wave_incl_max_dpp((in && g != gp) ? e : -1), carry);
        carry = readlane_i(s0, WAVE - 1);
        if (in) {
            const int64_t at = (int64_t)tptr[tile_table_off(g, K, rgs) + (k << rgs)] + (e - s0);
            if constexpr (MODE == 0) store_rec(rec, at, c & ((1 << tws) - 1), Bx[r0 + e]);
            else if constexpr (MODE == 1) store_rec_col<T>(rec, at, c & ((1 << tws) - 1));
            else tm[at] = Bx[r0 + e];
        }
    }
}

// Value parts of records [*lo, *hi) from the tile-major values (the bounds are segment-table
// words, read on the device: the host never waits for them).
template <typename T>
__global__ __launch_bounds__(256) void k_bt_fill(const int32_t* __restrict__ lo, const int32_t* __restrict__ hi,
                                                 const T* __restrict__ tm, uint32_t* __restrict__ rec) {
    const int64_t r0 = *lo, r1 = *hi;
    for (int64_t r = r0 + (int64_t)blockIdx.x * 256 + threadIdx.x; r < r1; r += (int64_t)gridDim.x * 256)
        store_rec_val<T>(rec, r, tm[r]);
}

// (start, end) of B row k's segment in a tile (tp = tptr + tile_table_off(g, ..)): two
// adjacent table words with one 8-byte load (4-byte aligned: one request instead of two)
__device__ __forceinline__ uint2 seg_pair(const int32_t* __restrict__ tp, int32_t k, int rgs) {
    uint2 v;
    __builtin_memcpy(&v, tp + ((int64_t)k << rgs), sizeof(v));
    return v;
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
    uint8_t mk[TILE_MK];
};

// Lane -> A-entry map for a group of up to 16 chunks (1024 products) starting at gbase.
// Marker byte l + 1 where A entry l's products start, 0 elsewhere, stored transposed: the
// marker of product t (group-relative) at byte 16 * (t % 64) + t / 64, so each lane reads
// the markers of all 16 chunks of its lane position with one 16-byte LDS load.  An
// unsigned max-scan over a chunk's 64 markers (identity 0: one v_max_u32_dpp per step)
// gives each lane its A entry + 1; `carry` (0 = none yet) brings it over from the previous
// chunk.
template <typename L>
__device__ __forceinline__ void group_markers(L& S, int l, int cnt, int off, int gbase) {
    wsync();
    reinterpret_cast<uint4*>(S.mk)[l] = make_uint4(0u, 0u, 0u, 0u);
    wsync();
    if (cnt > 0 && off >= gbase && off < gbase + TILE_MK) {
        const int t = off - gbase;
        S.mk[((t & (WAVE - 1)) << 4) | (t >> 6)] = (uint8_t)(l + 1);
    }
    wsync();
}

// The marker bytes of chunks cb .. cb+7 of this lane's 16 (cb a multiple of the chunks per
// step: 4 or 8), byte u = chunk cb + u.
__device__ __forceinline__ uint64_t marker_bytes(uint4 m, int cb) {
    const uint64_t lo = ((uint64_t)m.y << 32) | m.x, hi = ((uint64_t)m.w << 32) | m.z;
    if (cb == 0) return lo;
    if (cb >= 8) return hi >> (8 * (cb - 8));
    return (lo >> (8 * cb)) | (hi << (64 - 8 * cb));
}

// Chunks of one group (<= 16 x 64 products) U at a time: map lanes to A entries for U
// chunks, issue all their column loads, then hand each chunk to `fn(col)` in order (lanes
// past the group's products get col = -1).
template <int U, typename IP, typename CT, typename L, typename F>
__device__ __forceinline__ void walk_group(L& S, int l, int gb, int Pb, unsigned& carry,
                                           const CT* __restrict__ Bj, F&& fn) {
    const int nchg = min(TILE_MK, Pb - gb);
    const uint4 mrow = reinterpret_cast<const uint4*>(S.mk)[l];
    for (int c0 = 0; c0 < nchg; c0 += U * WAVE) {
        const uint64_t mb = marker_bytes(mrow, c0 >> 6);
        IP idx[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            idx[u] = (IP)-1;
            const int cc = c0 + u * WAVE;
            if (cc < nchg) {
                const unsigned sp = max(wave_incl_umax_dpp((unsigned)(mb >> (8 * u)) & 0xffu), carry);
                carry = (unsigned)readlane_i((int)sp, WAVE - 1);
                const int src = (int)sp - 1;
                const int t = gb + cc + l;
                if (t < Pb) idx[u] = S.jb0[src] + (IP)(t - (int)S.joff[src]);
            }
        }
        int col[U];
#pragma unroll
        for (int u = 0; u < U; ++u) col[u] = idx[u] >= 0 ? (int)Bj[idx[u]] : -1;
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (c0 + u * WAVE < nchg) fn(col[u]);
    }
}

// B's column indices modulo 65536, 2 bytes each: the symbolic passes read these instead of the
// 4-byte indices (half the bytes of the column gathers).  A symbolic tile is at most 65536
// columns wide and aligned to its width, so it never crosses a 65536-aligned block and a
// column's offset inside it is (col & 0xffff) - (lo & 0xffff).
__global__ __launch_bounds__(256) void k_bj16(int64_t nnz, const int32_t* __restrict__ Bj, uint16_t* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nnz; i += (int64_t)gridDim.x * 256)
        out[i] = (uint16_t)(Bj[i] & 0xffff);
}

// Symbolic pass of the tile path over wide symbolic tiles: R = 2^(twss - tws) numeric
// tiles at once (up to 65536 columns, the whole row for N <= 65536), so B rows are read in
// long coalesced segments.  Writes each numeric tile's bitmap (contiguous per row) and its
// entry count.  Columns come from Bj16 (k_bj16).
template <typename IP>
__global__ __launch_bounds__(TILE_WPB * WAVE) void k_tile_sym(
    int64_t row0, int64_t nrows, int tws, int G, int twss, const IP* __restrict__ Ap,
    const int32_t* __restrict__ Aj, const IP* __restrict__ Bp, const uint16_t* __restrict__ Bj16,
    const uint32_t* __restrict__ sidx, uint32_t* __restrict__ bitmap, int64_t* __restrict__ item_cnt) {
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
        const int lo16 = (t0 << tws) & 0xffff;   // the tile's start inside its 65536-column block
        const int nws = (t1 - t0) * nw;
        const int64_t a0 = Ap[row];
        const int nA = (int)(Ap[row + 1] - a0);
        if (nA <= 0) {
            for (int t = t0 + l; t < t1; t += WAVE) item_cnt[(row - row0) * G + t] = 0;
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
                    const uint32_t* sk = sidx + (int64_t)k * (Gs + 1);
                    const uint32_t s0 = sk[gs];
                    cnt = (int)(sk[gs + 1] - s0);
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
            unsigned carry = 0u;
            for (int gb = 0; gb < Pb; gb += TILE_MK) {
                group_markers(S, l, cnt, off, gb);
                walk_group<8, IP>(S, l, gb, Pb, carry, Bj16, [&](int c) {
                    if (c >= 0) set_bit(S.bits, c - lo16);
                });
            }
        }
        wsync();
        if (bitmap) {   // (dense numeric tiles take their structure from the accumulation)
            uint32_t* __restrict__ out = bitmap + ((row - row0) * G + t0) * (int64_t)nw;
            for (int w = l; w < nws; w += WAVE) out[w] = S.bits[w];
        }
        // entry count of each numeric tile: lane t sums tile t's words (rotated start: no
        // two lanes read one bank together)
        for (int t = l; t < t1 - t0; t += WAVE) {
            int c = 0;
            for (int j = 0; j < nw; ++j) c += __popc(S.bits[t * nw + ((j + t) & (nw - 1))]);
            item_cnt[(row - row0) * G + t0 + t] = c;
        }
    }
}

// Symbolic pass of the tile path, walking 16-byte WORDS of B's 16-bit columns (k_bj16) instead
// of products (round 4).  The bitmap OR is order-free, so a wave needs no (jj, kk) product order:
// each A entry's segment [beg, beg + cnt) of its B row inside the symbolic tile covers
// ceil(((beg & 7) + cnt) / 8) aligned words; the words of a batch of 64 entries are flattened
// (DPP scan of the word counts, transposed markers + max-scan for the lane -> entry map, as
// k_tile_sym does for products) and every lane loads ONE word -- 8 columns -- per chunk of 64
// words, masks the columns outside its entry's segment and sets their bits.  A chunk thus moves
// up to 512 columns with one 16-byte load per lane where k_tile_sym moves 64 with one 2-byte load
// per lane (config 5's 65-column segments: ~9 words each, 89 % of the slots used).
struct __attribute__((aligned(16))) Sym8Ent {
    uint32_t w0;     // first word (index into the uint4 view of Bj16)
    uint32_t woff;   // flattened offset of the entry's first word
    uint32_t wlen;   // words
    uint32_t lohi;   // (beg & 7) | (((beg + cnt - 1) & 7) + 1) << 8: valid halves of the first / last word
};
#ifndef SPG_SYM_MAXLOG
#define SPG_SYM_MAXLOG 16   // (A/B: a narrower cap on the k_tile_sym8 tile, spgemm.hip sym_tile_log2)
#endif
constexpr int SYM8_NW = 1 << (SPG_SYM_MAXLOG - 5);   // k_tile_sym8 bitmap words (the widest tile)
struct Sym8Lds {
    uint32_t bits[SYM8_NW];
    Sym8Ent ent[WAVE];
    uint8_t mk[TILE_MK];
};
#ifndef SPG_SYM8_WPE
#define SPG_SYM8_WPE 1   // (A/B: a waves-per-SIMD floor for k_tile_sym8's register budget)
#endif
template <typename IP>
__global__ __launch_bounds__(TILE_WPB * WAVE) __attribute__((amdgpu_waves_per_eu(SPG_SYM8_WPE))) void k_tile_sym8(
    int64_t row0, int64_t nrows, int tws, int G, int twss, const IP* __restrict__ Ap,
    const int32_t* __restrict__ Aj, const IP* __restrict__ Bp, const uint16_t* __restrict__ Bj16,
    const uint32_t* __restrict__ sidx, uint32_t* __restrict__ bitmap, int64_t* __restrict__ item_cnt) {
    constexpr int U = 8;   // chunks of 64 words in flight
    __shared__ __attribute__((aligned(16))) Sym8Lds lds[TILE_WPB];
    const int l = lane_id();
    const int wv = uniform((int)(threadIdx.x >> 6));
    Sym8Lds& S = lds[wv];
    const uint4* __restrict__ W = reinterpret_cast<const uint4*>(Bj16);
    const int nw = (1 << tws) >> 5;           // bitmap words of a numeric tile
    const int R = 1 << (twss - tws);          // numeric tiles per symbolic tile
    const int Gs = (G + R - 1) / R;           // symbolic tiles per row
    const uint32_t tasks = (uint32_t)(nrows * Gs);
    const uint32_t stride = gridDim.x * TILE_WPB;
    for (uint32_t task = xcd_block(gridDim.x) * TILE_WPB + wv; task < tasks; task += stride) {
        const int64_t row = row0 + (int64_t)(task / (uint32_t)Gs);
        const int gs = (int)(task % (uint32_t)Gs);
        const int t0 = gs * R, t1 = min(G, t0 + R);
        const int lo16 = (t0 << tws) & 0xffff;
        const int nws = (t1 - t0) * nw;
        const int64_t a0 = Ap[row];
        const int nA = (int)(Ap[row + 1] - a0);
        if (nA <= 0) {
            for (int t = t0 + l; t < t1; t += WAVE) item_cnt[(row - row0) * G + t] = 0;
            continue;
        }
        wsync();
        for (int w = l; w < nws; w += WAVE) S.bits[w] = 0u;
        for (int b = 0; b < nA; b += WAVE) {
            int wlen = 0;
            Sym8Ent e{0u, 0u, 0u, 0u};
            int64_t bg = 0;
            int cnt = 0;
            if (b + l < nA) {
                const int32_t k = Aj[a0 + b + l];
                const IP rb = Bp[k];
                if (Gs == 1) {
                    cnt = (int)(Bp[k + 1] - rb);
                    bg = (int64_t)rb;
                } else {
                    const uint32_t* sk = sidx + (int64_t)k * (Gs + 1);
                    const uint32_t s0 = sk[gs];
                    cnt = (int)(sk[gs + 1] - s0);
                    bg = (int64_t)rb + s0;
                }
            }
            if (cnt > 0) {
                wlen = (int)(((bg + cnt + 7) >> 3) - (bg >> 3));
                e.w0 = (uint32_t)(bg >> 3);
                e.lohi = (uint32_t)(bg & 7) | ((uint32_t)(((bg + cnt - 1) & 7) + 1) << 8);
            }
            const int incl = wave_incl_sum_dpp(wlen);
            const int woff = incl - wlen;
            const int Wb = readlane_i(incl, WAVE - 1);
            wsync();
            e.woff = (uint32_t)woff;
            e.wlen = (uint32_t)wlen;
            S.ent[l] = e;
            wsync();
            unsigned carry = 0u;
            for (int gb = 0; gb < Wb; gb += TILE_MK) {
                group_markers(S, l, wlen, woff, gb);
                const int nchg = min(TILE_MK, Wb - gb);
                const uint4 mrow = reinterpret_cast<const uint4*>(S.mk)[l];
                for (int c0 = 0; c0 < nchg; c0 += U * WAVE) {
                    const uint64_t mb = marker_bytes(mrow, c0 >> 6);
                    uint4 w[U];
                    uint32_t lo[U], hi[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        lo[u] = 8u;   // (no valid column: slots past the group's words)
                        hi[u] = 0u;
                        w[u] = make_uint4(0u, 0u, 0u, 0u);
                        const int cc = c0 + u * WAVE;
                        if (cc < nchg) {
                            const unsigned sp = max(wave_incl_umax_dpp((unsigned)(mb >> (8 * u)) & 0xffu), carry);
                            carry = (unsigned)readlane_i((int)sp, WAVE - 1);
                            const int t = gb + cc + l;
                            if (t < Wb) {
                                const Sym8Ent x = S.ent[(int)sp - 1];
                                const uint32_t wi = (uint32_t)t - x.woff;
                                lo[u] = wi == 0u ? (x.lohi & 0xffu) : 0u;
                                hi[u] = wi + 1u == x.wlen ? (x.lohi >> 8) : 8u;
                                w[u] = W[x.w0 + wi];
                            }
                        }
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint32_t ww[4] = {w[u].x, w[u].y, w[u].z, w[u].w};
#pragma unroll
                        for (int h = 0; h < 8; ++h)
                            if ((uint32_t)h >= lo[u] && (uint32_t)h < hi[u])
                                set_bit(S.bits, (int)((ww[h >> 1] >> (16 * (h & 1))) & 0xffffu) - lo16);
                    }
                }
            }
        }
        wsync();
        if (bitmap) {   // (dense numeric tiles take their structure from the accumulation)
            uint32_t* __restrict__ out = bitmap + ((row - row0) * G + t0) * (int64_t)nw;
            for (int w = l; w < nws; w += WAVE) out[w] = S.bits[w];
        }
        for (int t = l; t < t1 - t0; t += WAVE) {
            int c = 0;
            for (int j = 0; j < nw; ++j) c += __popc(S.bits[t * nw + ((j + t) & (nw - 1))]);
            item_cnt[(row - row0) * G + t0 + t] = c;
        }
    }
}

// SPG_SYM8_PF (round 6): k_tile_sym8c loads the next batch's extents during the current batch
// (config 5 symbolic 12.0 -> 11.5 ms; 0: round 5's per-batch dependent chain)
#ifndef SPG_SYM8_PF
#define SPG_SYM8_PF 1
#endif
#ifndef SPG_SYM8_U
#define SPG_SYM8_U 8   // (A/B: chunks of 64 words in flight in k_tile_sym8c)
#endif
// k_tile_sym8 with CW waves per task (round 5): the task's bitmap is shared in LDS by the
// block's waves (the bitmap OR is order-free: ds_or from any wave), each wave walks every CW-th
// batch of 64 A entries with its own entry table and markers.  The 8 KB bitmap is then paid once
// per CW waves: 12 KB per 2-wave block instead of 20 KB, so a CU holds 24 waves instead of 16
// (config 5's symbolic pass was waiting on memory with 4 waves per SIMD).
struct Sym8Wave {
    Sym8Ent ent[WAVE];
    uint8_t mk[TILE_MK];
};
template <int CW> struct Sym8Blk {
    uint32_t bits[SYM8_NW];
    Sym8Wave w[CW];
};
template <typename IP, int CW>
__global__ __launch_bounds__(CW * WAVE) void k_tile_sym8c(
    int64_t row0, int64_t nrows, int tws, int G, int twss, const IP* __restrict__ Ap,
    const int32_t* __restrict__ Aj, const IP* __restrict__ Bp, const uint16_t* __restrict__ Bj16,
    const uint32_t* __restrict__ sidx, uint32_t* __restrict__ bitmap, int64_t* __restrict__ item_cnt) {
    constexpr int U = SPG_SYM8_U;   // chunks of 64 words in flight
    constexpr int NT = CW * WAVE;
    __shared__ __attribute__((aligned(16))) Sym8Blk<CW> blk;
    const int l = lane_id();
    const int tid = (int)threadIdx.x;
    const int wv = uniform(tid >> 6);
    Sym8Wave& S = blk.w[wv];
    uint32_t* bits = blk.bits;
    const uint4* __restrict__ W = reinterpret_cast<const uint4*>(Bj16);
    const int nw = (1 << tws) >> 5;           // bitmap words of a numeric tile
    const int R = 1 << (twss - tws);          // numeric tiles per symbolic tile
    const int Gs = (G + R - 1) / R;           // symbolic tiles per row
    const uint32_t tasks = (uint32_t)(nrows * Gs);
    for (uint32_t task = xcd_block(gridDim.x); task < tasks; task += gridDim.x) {
        __syncthreads();   // (the previous task's bitmap has been written out)
        const int64_t row = row0 + (int64_t)(task / (uint32_t)Gs);
        const int gs = (int)(task % (uint32_t)Gs);
        const int t0 = gs * R, t1 = min(G, t0 + R);
        const int lo16 = (t0 << tws) & 0xffff;
        const int nws = (t1 - t0) * nw;
        const int64_t a0 = Ap[row];
        const int nA = (int)(Ap[row + 1] - a0);
        if (nA <= 0) {
            for (int t = t0 + tid; t < t1; t += NT) item_cnt[(row - row0) * G + t] = 0;
            continue;
        }
        for (int w = tid; w < nws; w += NT) bits[w] = 0u;
        __syncthreads();
        // SPG_SYM8_PF (round 6): the next batch's extents (A column -> B row start and, for a
        // row cut into symbolic tiles, the tile's bounds) are loaded during this batch, as raw
        // words (unconditional loads at a clamped entry; nothing waits for them until the next
        // batch starts) -- one dependent chain of three loads per batch no longer stalls it
        // (specialised for whole-row symbolic tiles, Gs == 1: no uniform branch between a load
        // and its use)
        auto batches = [&](auto gs1) {
            IP xr = 0, xe = 0;
            uint32_t xs0 = 0u, xs1 = 0u;
            auto fetch = [&](int bn) {
                const int32_t k = Aj[a0 + min(bn + l, nA - 1)];
                xr = Bp[k];
                if constexpr (decltype(gs1)::value) {
                    xe = Bp[k + 1];
                } else {
                    const uint32_t* sk = sidx + (int64_t)k * (Gs + 1);
                    xs0 = sk[gs];
                    xs1 = sk[gs + 1];
                }
            };
            if (SPG_SYM8_PF) fetch(wv * WAVE);
            for (int b = wv * WAVE; b < nA; b += NT) {
                int wlen = 0;
                Sym8Ent e{0u, 0u, 0u, 0u};
                int64_t bg = 0;
                int cnt = 0;
                if (SPG_SYM8_PF) {
                    if (b + l < nA) {
                        if constexpr (decltype(gs1)::value) {
                            cnt = (int)(xe - xr);
                            bg = (int64_t)xr;
                        } else {
                            cnt = (int)(xs1 - xs0);
                            bg = (int64_t)xr + xs0;
                        }
                    }
                    fetch(b + NT);   // (unconditional: a conditional load would make the compiler wait for it)
                } else if (b + l < nA) {
                    const int32_t k = Aj[a0 + b + l];
                    const IP rb = Bp[k];
                    if (Gs == 1) {
                        cnt = (int)(Bp[k + 1] - rb);
                        bg = (int64_t)rb;
                    } else {
                        const uint32_t* sk = sidx + (int64_t)k * (Gs + 1);
                        const uint32_t s0 = sk[gs];
                        cnt = (int)(sk[gs + 1] - s0);
                        bg = (int64_t)rb + s0;
                    }
                }
                if (cnt > 0) {
                    wlen = (int)(((bg + cnt + 7) >> 3) - (bg >> 3));
                    e.w0 = (uint32_t)(bg >> 3);
                    e.lohi = (uint32_t)(bg & 7) | ((uint32_t)(((bg + cnt - 1) & 7) + 1) << 8);
                }
                const int incl = wave_incl_sum_dpp(wlen);
                const int woff = incl - wlen;
                const int Wb = readlane_i(incl, WAVE - 1);
                wsync();
                e.woff = (uint32_t)woff;
                e.wlen = (uint32_t)wlen;
                S.ent[l] = e;
                wsync();
                unsigned carry = 0u;
                for (int gb = 0; gb < Wb; gb += TILE_MK) {
                    group_markers(S, l, wlen, woff, gb);
                    const int nchg = min(TILE_MK, Wb - gb);
                    const uint4 mrow = reinterpret_cast<const uint4*>(S.mk)[l];
                    for (int c0 = 0; c0 < nchg; c0 += U * WAVE) {
                        const uint64_t mb = marker_bytes(mrow, c0 >> 6);
                        const uint64_t mb2 = U > 8 ? marker_bytes(mrow, (c0 >> 6) + 8) : 0ull;   // (chunks 8..15 of a 16-chunk step)
                        uint4 w[U];
                        uint32_t lo[U], hi[U];
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            lo[u] = 8u;   // (no valid column: slots past the group's words)
                            hi[u] = 0u;
                            w[u] = make_uint4(0u, 0u, 0u, 0u);
                            const int cc = c0 + u * WAVE;
                            if (cc < nchg) {
                                const unsigned sp = max(wave_incl_umax_dpp((unsigned)((u < 8 ? mb : mb2) >> (8 * (u & 7))) & 0xffu), carry);
                                carry = (unsigned)readlane_i((int)sp, WAVE - 1);
                                const int t = gb + cc + l;
                                if (t < Wb) {
                                    const Sym8Ent x = S.ent[(int)sp - 1];
                                    const uint32_t wi = (uint32_t)t - x.woff;
                                    lo[u] = wi == 0u ? (x.lohi & 0xffu) : 0u;
                                    hi[u] = wi + 1u == x.wlen ? (x.lohi >> 8) : 8u;
                                    w[u] = W[x.w0 + wi];
                                }
                            }
                        }
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            const uint32_t ww[4] = {w[u].x, w[u].y, w[u].z, w[u].w};
#pragma unroll
                            for (int h = 0; h < 8; ++h)
                                if ((uint32_t)h >= lo[u] && (uint32_t)h < hi[u])
                                    set_bit(bits, (int)((ww[h >> 1] >> (16 * (h & 1))) & 0xffffu) - lo16);
                        }
                    }
                }
            }
        };
        if (Gs == 1) batches(std::true_type{});
        else batches(std::false_type{});
        __syncthreads();
        if (bitmap) {   // (dense numeric tiles take their structure from the accumulation)
            uint32_t* __restrict__ out = bitmap + ((row - row0) * G + t0) * (int64_t)nw;
            for (int w = tid; w < nws; w += NT) out[w] = bits[w];
        }
        for (int t = tid; t < t1 - t0; t += NT) {
            int c = 0;
            for (int j = 0; j < nw; ++j) c += __popc(bits[t * nw + ((j + t) & (nw - 1))]);
            item_cnt[(row - row0) * G + t0 + t] = c;
        }
    }
}

// Numeric pass of the tile path: one wave per item (row, numeric tile).  Reads the item's
// bitmap from the symbolic pass, enumerates its products in flattened (jj, kk) order --
// two adjacent 4-byte loads from tile g's segment table per A entry, one record load per
// product from tile g's slice of the tile-major B -- and accumulates lowest-lane-first per
// output position.  Items are taken tile-major (item = g * nrows + row) and the XCD-aware
// block map gives every XCD a contiguous run of them: an XCD works through one tile at a
// time, so the tile's B slice and segment table stay in its L2, while the eight XCDs sweep
// the A rows in the same order (an A row comes from HBM about once per eight tiles, the
// other reads hit the Infinity Cache).
//
// Positions: DENSE (tile width <= CAP, one window) addresses the accumulator by column
// (c - lo); otherwise by the popcount prefix of the symbolic bitmap, in column windows of
// <= CAP entries (products re-read per window).
// Ordered adds: products are taken U chunks (U * 64) at a time, all their record loads in
// flight; then groups of RU chunks resolve collisions in owner rounds: a ds_min of the key
// (round, chunk, lane) per product, the product whose key stuck adds, the others retry with
// the next (smaller) round number.  Within a group the lowest (chunk, lane) -- the earliest
// product in flattened order -- of every position adds first; groups run in order.
// Timing-only diagnostics of k_tile (results WRONG; A/B timing builds only, never shipped):
// 1 = no accumulation, 2 = no record loads, 4 = no product batches, 8 = no output stores.
#ifndef SPG_TILE_DIAG
#define SPG_TILE_DIAG 0
#endif

template <typename T, typename IP, bool DENSE, int RU>
__global__ __launch_bounds__(tile_num_wpb<DENSE>() * WAVE) void k_tile(
    int64_t row0, int64_t nrows, int tws, int G, const IP* __restrict__ Ap,
    const int32_t* __restrict__ Aj, const T* __restrict__ Ax, int64_t K,
    const uint32_t* __restrict__ brec, const int32_t* __restrict__ tptr,
    const uint32_t* __restrict__ bitmap, const int64_t* __restrict__ item_off,
    int32_t* __restrict__ Cj, T* __restrict__ Cx, T alpha, uint32_t it_lo, uint32_t it_hi, int rgs) {
    constexpr int diag = SPG_TILE_DIAG;   // 0 in every shipped build (timing-only diagnostics)
    constexpr int U = sizeof(T) > 8 ? 4 : 8;   // chunks in flight (complex128: half)
    static_assert(U % RU == 0, "round groups split the chunks in flight");
    constexpr int WPB = tile_num_wpb<DENSE>();
    __shared__ __attribute__((aligned(16))) NumLds<T, IP, DENSE> lds[WPB];
    const int l = lane_id();
    const int wv = uniform((int)(threadIdx.x >> 6));
    NumLds<T, IP, DENSE>& S = lds[wv];
    const int TW = 1 << tws;
    const int nw = TW >> 5;                    // bitmap words of a tile
    const int wpl = (nw + WAVE - 1) / WAVE;    // words per lane (<= 2)
    // items [it_lo, it_hi) (tile-major: a range of whole tiles; rows*G < 2^31 on the host)
    for (uint32_t it = it_lo + xcd_block(gridDim.x) * WPB + wv; it < it_hi; it += gridDim.x * WPB) {
        const int g = (int)(it / (uint32_t)nrows);
        const int64_t row = row0 + (int64_t)(it - (uint32_t)g * (uint32_t)nrows);
        const int64_t item = (row - row0) * G + g;   // items (and bitmaps) of this chunk of rows
        const int32_t* __restrict__ tp = tptr + tile_table_off(g, K, rgs);   // tile g's segment table
        const int lo = g * TW;
        const int64_t a0 = Ap[row];
        const int nA = (int)(Ap[row + 1] - a0);
        if (nA <= 0) continue;
        // the item's entries: DENSE from its offsets (its structure comes from the
        // accumulation tags below); otherwise the symbolic bitmap and its popcount prefix
        // (lane owns wpl words)
        const int w0 = min(nw, l * wpl), w1 = min(nw, w0 + wpl);
        int nnz, pincl = 0, p0 = 0;
        if constexpr (DENSE) {
            nnz = (int)(item_off[item + 1] - item_off[item]);
            if (nnz == 0) continue;
        } else {
            const uint32_t* __restrict__ ibits = bitmap + item * nw;
            uint32_t wd[2] = {0u, 0u};
            int mine = 0;
#pragma unroll
            for (int q = 0; q < 2; ++q)
                if (w0 + q < w1) {
                    wd[q] = ibits[w0 + q];
                    mine += __popc(wd[q]);
                }
            pincl = wave_incl_sum_dpp(mine);
            nnz = readlane_i(pincl, WAVE - 1);
            if (nnz == 0) continue;
            p0 = pincl - mine;
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
        }
        const int64_t obase = item_off[item];
        // The first NB batches of A entries (rows of <= NB*64 entries: all of them): every
        // lane's A entry, value and tile segment, loaded at once up front (two dependent
        // load levels per item instead of two per batch).
        constexpr int NB = sizeof(T) > 8 ? 4 : 8;
        int32_t kq[NB];
        T aq[NB];
        uint2 sq[NB];
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
            if (kq[q] >= 0) sq[q] = seg_pair(tp, kq[q], rgs);
        }
        // lane info of one batch of A entries: (first B index, count) of its tile segment
        auto batch = [&](int b, int& cnt, int& off, int& Pb, T& bav) {
            cnt = 0;
            IP beg = 0;
            T av = (T)0;
            if (b < NB * WAVE) {
#pragma unroll
                for (int q = 0; q < NB; ++q)
                    if (q == (b >> 6)) {
                        cnt = (int)(sq[q].y - sq[q].x);
                        beg = (IP)sq[q].x;
                        av = aq[q];
                    }
            } else if (b + l < nA) {
                const uint2 se = seg_pair(tp, Aj[a0 + b + l], rgs);
                cnt = (int)(se.y - se.x);
                beg = (IP)se.x;
                av = Ax[a0 + b + l];
            }
            const int incl = wave_incl_sum_dpp(cnt);
            off = incl - cnt;
            Pb = readlane_i(incl, WAVE - 1);
            wsync();
            S.ent[l] = TileSeg<IP>{beg, (uint32_t)off};
            bav = av;
            wsync();
        };
        for (int L0 = 0; L0 < WAVE;) {
            int L1 = WAVE, wb = 0, wn = nnz;
            if (!DENSE && nnz > TILE_CAP) {
                wb = readlane_i(p0, L0);
                L1 = (int)__popcll(__ballot(pincl <= wb + TILE_CAP));
                if (L1 <= L0) L1 = L0 + 1;
                wn = (L1 < WAVE ? readlane_i(p0, L1) : nnz) - wb;
            }
            const int clo = 32 * wpl * L0, chi = 32 * wpl * L1;   // window, tile-relative
            const int span = DENSE ? TW : wn;   // accumulator slots in use
            if constexpr (DENSE) {   // 16-byte stores (TW is a multiple of 64)
                uint4* a4 = reinterpret_cast<uint4*>(S.acc);
                uint4* t4 = reinterpret_cast<uint4*>(S.tag);
                for (int q = l; q < TW * (int)sizeof(T) / 16; q += WAVE) a4[q] = make_uint4(0u, 0u, 0u, 0u);
                for (int q = l; q < TW / 4; q += WAVE) t4[q] = make_uint4(~0u, ~0u, ~0u, ~0u);
            } else {
                for (int p = l; p < span; p += WAVE) {
                    S.acc[p] = (T)0;
                    S.tag[p] = 0xffffffffu;
                }
            }
            wsync();
            // 23 bits: key = seq | chunk (3 bits) | lane (6 bits); every key < 0xfffffdff, so
            // a tag below 0xfffffffe marks a column some product reached (DENSE: the
            // item's structure)
            uint32_t seq = 0x7ffffeu;
            for (int b = 0; b < ((diag & 4) ? 0 : nA); b += WAVE) {   // (diag 4, timing only: no batches)
                int cnt, off, Pb;
                T bav;   // this lane's A value of the batch
                batch(b, cnt, off, Pb, bav);
                unsigned carry = 0u;
                for (int gb = 0; gb < Pb; gb += NUM_MK) {
                    num_group_markers(S, l, cnt, off, gb);
                    const int nchg = min(NUM_MK, Pb - gb);
                    const uint2 m2 = reinterpret_cast<const uint2*>(S.mk)[l];
                    const uint64_t mrow = ((uint64_t)m2.y << 32) | m2.x;
                    for (int c0 = 0; c0 < nchg; c0 += U * WAVE) {
                        // U, 3U/4 or U/2 chunks at once, the fewest that hold the group's
                        // remaining products (a wave-uniform choice: short batches scan and
                        // load few empty slots)
                        const int nu = min(U, (nchg - c0 + WAVE - 1) >> 6);
                        auto step = [&](auto nuc) {
                            constexpr int NU = decltype(nuc)::value;
                            constexpr int RG = RU < NU ? RU : NU;
                            // NU chunks at once (nu of them hold products: a wave-uniform count):
                            // the lane -> A entry scans, then every record load in flight.
                            const uint64_t mb = mrow >> (8 * (c0 >> 6));
                            // (slots past nu scan zero markers and load record 0: no branches
                            // between the loads, so they all stay in flight)
                            unsigned sp[NU];
#pragma unroll
                            for (int u = 0; u < NU; ++u) sp[u] = wave_incl_umax_dpp((unsigned)(mb >> (8 * u)) & 0xffu);
#pragma unroll
                            for (int u = 0; u < NU; ++u) {
                                sp[u] = max(sp[u], carry);
                                carry = (unsigned)readlane_i((int)sp[u], WAVE - 1);
                            }
                            IP idx[NU];
                            T av[NU];
                            bool val[NU];
#pragma unroll
                            for (int u = 0; u < NU; ++u) {
                                const int t = gb + c0 + u * WAVE + l;
                                val[u] = u < nu && t < Pb;
                                const int src = (int)max(sp[u], 1u) - 1;
                                const TileSeg<IP> e = S.ent[src];
                                idx[u] = val[u] ? e.jb0 + (IP)(t - (int)e.joff) : (IP)0;
                                av[u] = shfl_v(bav, src);
                            }
                            int qc[NU];
                            T qv[NU];
                            if (diag & 2) {   // timing only: no record loads
#pragma unroll
                                for (int u = 0; u < NU; ++u) { qc[u] = (int)((idx[u] * 37u) & (uint32_t)(TW - 1)); qv[u] = (T)1; }
                            } else {
#pragma unroll
                                for (int u = 0; u < NU; ++u) load_rec(brec, idx[u], qc[u], qv[u]);
                            }
                            int pos[NU];
                            T pv[NU];
                            uint32_t pend = 0u;
#pragma unroll
                            for (int u = 0; u < NU; ++u) {
                                pos[u] = 0;
                                pv[u] = (T)0;
                                {
                                    const int rc = val[u] ? qc[u] : -1;   // column inside the tile
                                    if constexpr (DENSE) {
                                        if (rc >= 0) {
                                            pos[u] = rc;
                                            pend |= 1u << u;
                                        }
                                    } else if (rc >= clo && rc < chi) {
                                        const uint2 bw = S.bw[rc >> 5];
                                        pos[u] = (int)bw.y + __popc(bw.x & ((1u << (rc & 31)) - 1u)) - wb;
                                        pend |= 1u << u;
                                    }
                                    pv[u] = mul_rn(av[u], qv[u]);
                                }
                            }
                            if (diag & 1) pend = 0u;   // timing only: no accumulation
#pragma unroll
                            for (int u0 = 0; u0 < NU; u0 += RG) {
                                uint32_t gm = pend & (((1u << RG) - 1u) << u0);
                                while (__ballot(gm != 0u)) {
                                    const uint32_t kb = (seq << 9) | (uint32_t)l;
#pragma unroll
                                    for (int u = u0; u < u0 + RG && u < NU; ++u)
                                        if (gm & (1u << u)) atomicMin(&S.tag[pos[u]], kb | ((uint32_t)u << 6));
#pragma unroll
                                    for (int u = u0; u < u0 + RG && u < NU; ++u)
                                        if ((gm & (1u << u)) &&
                                            __hip_atomic_load(&S.tag[pos[u]], __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_WAVEFRONT) == (kb | ((uint32_t)u << 6))) {
                                            S.acc[pos[u]] = add_rn(S.acc[pos[u]], pv[u]);
                                            gm &= ~(1u << u);
                                        }
                                    --seq;
                                }
                            }
                        };
                        if (nu > 3 * U / 4) step(std::integral_constant<int, U>{});
                        else if (nu > U / 2) step(std::integral_constant<int, 3 * U / 4>{});
                        else step(std::integral_constant<int, U / 2>{});
                        if (seq < 4096u) {   // re-arm the tag space (very long items only), keeping
                            wsync();          // which columns were reached (0xfffffffe)
                            for (int p = l; p < span; p += WAVE)
                                S.tag[p] = S.tag[p] == 0xffffffffu ? 0xffffffffu : 0xfffffffeu;
                            seq = 0x7ffffeu;
                            wsync();
                        }
                    }
                }
            }
            wsync();
            if constexpr (DENSE) {
                // the item's structure from the tags, 64 columns at a time: lane l looks at
                // column 64k + l; a column some product reached is an entry, its output
                // position the entries before it (the ballot's lower lanes plus the run)
                int32_t* __restrict__ crow = Cj + obase;
                T* __restrict__ xrow = Cx + obase;
                int run = 0;
                for (int k = 0; k < TW / WAVE; ++k) {
                    const int c = k * WAVE + l;
                    const bool hit = S.tag[c] != 0xffffffffu;
                    const unsigned long long m = __ballot(hit);
                    if (hit && !(diag & 8)) {   // (diag 8, timing only: no output)
                        const int p = run + lane_rank(m);
                        crow[p] = lo + c;
                        const T val = S.acc[c];
                        xrow[p] = (alpha == (T)1) ? val : mul_rn(alpha, val);
                    }
                    run += (int)__popcll(m);
                }
                wsync();
                break;
            }
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
                const uint32_t c = S.tag[p];
                const T val = S.acc[p];
                crow[p] = (int32_t)c;
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
