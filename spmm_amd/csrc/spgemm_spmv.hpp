// spgemm_spmv.hpp -- y = alpha * A x + beta * y for CSR A and dense x, y (the SpMV half of
// the reference's SpGEMM_vs_SpMV comparison, SpGEMM_vs_SpMV/profiler.py:410-411, reached
// through cupyx.cusparse.spmv, modify_src/cupy-src/cupyx/cusparse.py:1373-1432).
//
// Bit-identical to scipy's csr_matvec: every row is summed sequentially in A's entry order
// from 0 (((0 + a0 x0) + a1 x1) + ...), products and sums separately rounded.  To keep the
// loads coalesced anyway, a wave takes 64 consecutive rows: lanes form the products of the
// rows' contiguous entry range (Aj, Ax coalesced, x gathered) into LDS in entry order, then
// each lane sums its own row's products in order.  Long ranges go in chunks of SPMV_CH.
#pragma once

#include "spg_device.hpp"

namespace spg {

constexpr int SPMV_WPB = 4;
constexpr int SPMV_CH = 1024;   // products staged per wave per chunk

template <typename T, typename IP>
__global__ __launch_bounds__(SPMV_WPB * WAVE) void k_spmv(int64_t rows, const IP* __restrict__ Ap,
                                                        const int32_t* __restrict__ Aj,
                                                        const T* __restrict__ Ax, const T* __restrict__ x,
                                                        T alpha, T beta, T* __restrict__ y) {
    __shared__ T prod_s[SPMV_WPB][SPMV_CH];
    const int l = lane_id();
    const int wv = uniform((int)(threadIdx.x >> 6));
    T* prod = prod_s[wv];
    const int64_t r0 = ((int64_t)blockIdx.x * SPMV_WPB + wv) * WAVE;
    if (r0 >= rows) return;
    const int64_t r1 = min(rows, r0 + WAVE);
    const int64_t row = r0 + l;
    const int64_t a = row < rows ? (int64_t)Ap[row] : 0;
    const int64_t b = row < rows ? (int64_t)Ap[row + 1] : 0;
    const int64_t e0 = (int64_t)Ap[r0], e1 = (int64_t)Ap[r1];
    T sum = (T)0;
    for (int64_t c = e0; c < e1; c += SPMV_CH) {
        const int64_t ce = min(e1, c + SPMV_CH);
        for (int64_t e = c + l; e < ce; e += WAVE) prod[e - c] = mul_rn(Ax[e], x[Aj[e]]);
        wsync();
        const int64_t lo = max(a, c), hi = min(b, ce);
        for (int64_t e = lo; e < hi; ++e) sum = add_rn(sum, prod[e - c]);
        wsync();
    }
    if (row < rows) {
        T v = alpha == (T)1 ? sum : mul_rn(alpha, sum);
        if (beta != (T)0) v = add_rn(v, mul_rn(beta, y[row]));
        y[row] = v;
    }
}

}  // namespace spg
