// spg_device.hpp -- device-side building blocks of the gfx950 SpGEMM engine.
//
// Row-wise Gustavson (the same rule as scipy csr_matmat, restated in oracle/gustavson.c):
// output row i of C = sum over A's row-i entries (in stored order jj) of A[i,jj] * B[Aj[jj], :].
// One 64-lane wavefront owns one output row.  The row's columns are processed in column
// windows [lo, hi); per window the wave keeps, in its private slice of LDS:
//
//   bits[w]   one bit per column of the window (structure),
//   wpre[w]   exclusive popcount prefix of bits[] (column -> compact position),
//   acc[p]    the running sum of compact position p (sorted column order),
//   tag[p]    owner tags for ordered accumulation (re-used as the column list on output),
//   marker[]  64-entry scratch for mapping flattened product ids to A entries.
//
// Pass A (structure) sets bits; a popcount scan turns them into positions (this is the
// "wavefront segmented-scan row compression": positions come out in column order, so C
// needs no sort).  Pass B (values) enumerates the window's products in (jj, kk) order, 64
// at a time across the lanes, and adds each into acc[pos].  Two products of one 64-wide
// step may hit the same column (they come from different A entries); the lowest lane --
// the earlier product -- always goes first (owner rounds with ds_min on tag[]), so every
// C(i,j) is summed in exactly scipy's order with separately rounded mul/add.  No global
// atomics, no floating-point atomics: results are bit-reproducible.
//
// Windows: a row whose whole column range fits one window (<= NWMAX*32 columns and at
// most CAP structural entries) is done in one window with no searching.  Otherwise the
// columns are cut into windows sized so the expected entries fit CAP; per A entry the wave
// keeps a cursor into its (sorted) B row in a global scratch array and walks it window by
// window.  A window that still overflows CAP is halved and redone.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace spg {

constexpr int WAVE = 64;

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Compiler + wave-scope ordering point between LDS phases of one wave.  DS instructions
// of a wave execute in issue order on CDNA; this stops the compiler moving LDS accesses
// across the point (cross-lane communication through LDS is invisible to it).
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ int readlane_i(int v, int l) {
    return __builtin_amdgcn_readlane(v, l);
}

// Inclusive prefix sum over the 64 lanes.
__device__ __forceinline__ int wave_incl_sum(int v) {
    const int l = lane_id();
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
        int u = __shfl_up(v, d, WAVE);
        if (l >= d) v += u;
    }
    return v;
}

// lanes below this one whose bit of m is set
__device__ __forceinline__ int lane_rank(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

__device__ __forceinline__ long long wave_incl_sum64(long long v) {
    const int l = lane_id();
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
        long long u = __shfl_up(v, d, WAVE);
        if (l >= d) v += u;
    }
    return v;
}

// Inclusive prefix max over the 64 lanes.
__device__ __forceinline__ int wave_incl_max(int v) {
    const int l = lane_id();
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
        int u = __shfl_up(v, d, WAVE);
        if (l >= d) v = max(v, u);
    }
    return v;
}

__device__ __forceinline__ long long wave_sum64(long long v) {
#pragma unroll
    for (int d = WAVE / 2; d >= 1; d >>= 1) v += __shfl_xor(v, d, WAVE);
    return v;
}

// ---- DPP wave scans (gfx9 row_shr / row_bcast; no LDS traffic) ---------------------
// Inclusive prefix sum over the 64 lanes.
__device__ __forceinline__ int wave_incl_sum_dpp(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

// Inclusive prefix max over the 64 lanes for values >= -1.
__device__ __forceinline__ int wave_incl_max_dpp(int v) {
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x111, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x112, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x114, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x118, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x142, 0xa, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x143, 0xc, 0xf, false));
    return v;
}

// Inclusive prefix max over the 64 lanes for unsigned values.  0 is max_u32's identity, so
// each step folds into one v_max_u32_dpp (the signed form above needs a v_mov_b32_dpp too).
__device__ __forceinline__ unsigned wave_incl_umax_dpp(unsigned v) {
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
    return v;
}

__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Complex values (complex64 / complex128): two parts side by side, numpy's layout.  The
// default constructor is trivial, so the type can live in __shared__ arrays.
template <typename R> struct cplx {
    R re, im;
    cplx() = default;
    __host__ __device__ constexpr cplx(R r, R i) : re(r), im(i) {}
    __host__ __device__ constexpr cplx(int r) : re(R(r)), im(R(0)) {}   // (T)0, (T)1
};
template <typename R> __host__ __device__ inline bool operator==(cplx<R> a, cplx<R> b) {
    return a.re == b.re && a.im == b.im;
}
template <typename R> __host__ __device__ inline bool operator!=(cplx<R> a, cplx<R> b) { return !(a == b); }

// Separately rounded multiply and add (no contraction into FMA).  Complex products follow
// scipy's sparsetools complex_wrapper (and numpy): (ac - bd) + (ad + bc)i.
template <typename T> __device__ __forceinline__ T mul_rn(T a, T b);
template <> __device__ __forceinline__ double mul_rn<double>(double a, double b) { return __dmul_rn(a, b); }
template <> __device__ __forceinline__ float mul_rn<float>(float a, float b) { return __fmul_rn(a, b); }
template <> __device__ __forceinline__ cplx<double> mul_rn<cplx<double>>(cplx<double> a, cplx<double> b) {
    return cplx<double>(__dsub_rn(__dmul_rn(a.re, b.re), __dmul_rn(a.im, b.im)),
                        __dadd_rn(__dmul_rn(a.re, b.im), __dmul_rn(a.im, b.re)));
}
template <> __device__ __forceinline__ cplx<float> mul_rn<cplx<float>>(cplx<float> a, cplx<float> b) {
    return cplx<float>(__fsub_rn(__fmul_rn(a.re, b.re), __fmul_rn(a.im, b.im)),
                       __fadd_rn(__fmul_rn(a.re, b.im), __fmul_rn(a.im, b.re)));
}
template <typename T> __device__ __forceinline__ T add_rn(T a, T b);
template <> __device__ __forceinline__ double add_rn<double>(double a, double b) { return __dadd_rn(a, b); }
template <> __device__ __forceinline__ float add_rn<float>(float a, float b) { return __fadd_rn(a, b); }
template <> __device__ __forceinline__ cplx<double> add_rn<cplx<double>>(cplx<double> a, cplx<double> b) {
    return cplx<double>(__dadd_rn(a.re, b.re), __dadd_rn(a.im, b.im));
}
template <> __device__ __forceinline__ cplx<float> add_rn<cplx<float>>(cplx<float> a, cplx<float> b) {
    return cplx<float>(__fadd_rn(a.re, b.re), __fadd_rn(a.im, b.im));
}

// Lane shuffle of a value of any of the four value types.
template <typename T> __device__ __forceinline__ T shfl_v(T v, int s) { return __shfl(v, s, WAVE); }
template <typename R> __device__ __forceinline__ cplx<R> shfl_v(cplx<R> v, int s) {
    return cplx<R>(__shfl(v.re, s, WAVE), __shfl(v.im, s, WAVE));
}

// LDS footprint per wave.
template <typename T> struct NumGeom {
    static constexpr int BYTES = 16384;                 // per-wave LDS budget
    static constexpr int NWMAX = 512;                   // window <= 16384 columns
    static constexpr int CAP =
        (BYTES - NWMAX * 8 - WAVE * 4) / (int)(sizeof(T) + 4);   // entries per window
};

struct SymGeom {
    static constexpr int BYTES = 16384;
    static constexpr int NWMAX = (BYTES - WAVE * 4) / 4;         // 4032 words = 129024 cols
};

// Enumerate the products of one batch of up to 64 A entries (lane l <-> entry jj0+l) in
// flattened (jj, kk) order, 64 per step.  Each lane supplies `beg` (first B index of its
// segment) and `cnt` (segment length, 0 for an inactive lane).  For every step the functor
// is called uniformly with (valid, src_lane, idx): lane x handles product number
// step*64+x, which belongs to the A entry of lane `src_lane` and reads B entry `idx`.
template <typename F>
__device__ __forceinline__ void for_each_product(long long beg, int cnt, int* marker, F&& f) {
    const int l = lane_id();
    const int incl = wave_incl_sum(cnt);
    const int off = incl - cnt;
    const int total = readlane_i(incl, WAVE - 1);
    int carry = -1;
    for (int c0 = 0; c0 < total; c0 += WAVE) {
        marker[l] = -1;
        wsync();
        if (cnt > 0 && off >= c0 && off < c0 + WAVE) marker[off - c0] = l;
        wsync();
        int src = wave_incl_max(marker[l]);
        src = max(src, carry);
        carry = readlane_i(src, WAVE - 1);
        wsync();
        const int t = c0 + l;
        const bool valid = t < total;
        const int s = valid ? src : 0;
        const int soff = __shfl(off, s, WAVE);
        const long long sbeg = __shfl(beg, s, WAVE);
        f(valid, s, sbeg + (long long)(t - soff));
    }
}

// Exclusive popcount prefix of bits[0..nw) into wpre[]; returns the total (wave-uniform).
__device__ __forceinline__ int popcount_prefix(const uint32_t* bits, uint32_t* wpre, int nw) {
    const int l = lane_id();
    int base = 0;
    for (int w0 = 0; w0 < nw; w0 += WAVE) {
        const int w = w0 + l;
        const int c = (w < nw) ? __popc(bits[w]) : 0;
        const int incl = wave_incl_sum(c);
        if (w < nw) wpre[w] = (uint32_t)(base + incl - c);
        base += readlane_i(incl, WAVE - 1);
    }
    wsync();
    return base;
}

__device__ __forceinline__ void set_bit(uint32_t* bits, int rel) {
    atomicOr(&bits[rel >> 5], 1u << (rel & 31));
}

__device__ __forceinline__ int bit_pos(const uint32_t* bits, const uint32_t* wpre, int rel) {
    const int w = rel >> 5;
    const uint32_t m = (1u << (rel & 31)) - 1u;
    return (int)wpre[w] + __popc(bits[w] & m);
}

}  // namespace spg
