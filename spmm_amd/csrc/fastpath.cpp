// fastpath.cpp -- torch C++ extension: the allocation + call sequence of
// spmm_amd.cusparse.spgemm (cupyx.cusparse.spgemm, cupy-src/cupyx/cusparse.py:2041-2142) done
// natively, so a product costs one Python->C++ crossing instead of a dozen ctypes calls and
// tensor views.  It calls the same C ABI (libmi355_spgemm.so, include/spgemm.h) as the
// ctypes path; argument checking and the reference's exceptions stay in Python.
#include <torch/extension.h>

#include <cstdint>
#include <vector>

#include "spgemm.h"

namespace {

spg_index_t itype(const at::Tensor& t) { return t.scalar_type() == at::kLong ? SPG_INDEX_64I : SPG_INDEX_32I; }

spg_dtype_t vtype(const at::Tensor& t) {
    switch (t.scalar_type()) {
        case at::kFloat: return SPG_R_32F;
        case at::kDouble: return SPG_R_64F;
        case at::kComplexFloat: return SPG_C_32F;
        default: return SPG_C_64F;
    }
}

spg_csr_t view(int64_t rows, int64_t cols, const at::Tensor& p, const at::Tensor& j, const at::Tensor& x) {
    const int64_t nnz = x.numel();
    return spg_csr_t{rows, cols, nnz, p.data_ptr(), nnz ? j.data_ptr() : nullptr, nnz ? x.data_ptr() : nullptr,
                     itype(p), vtype(x)};
}

}  // namespace

// Returns (status, data, indices, indptr, workspace_bytes, peak_bytes).  status != 0: the
// tensors are undefined and the caller raises.
std::tuple<int64_t, at::Tensor, at::Tensor, at::Tensor, int64_t, int64_t> spgemm(
    int64_t handle, int64_t m, int64_t k, int64_t n, at::Tensor Ap, at::Tensor Aj, at::Tensor Ax, at::Tensor Bp,
    at::Tensor Bj, at::Tensor Bx, int64_t alg, double chunk_fraction, double alpha_re, double alpha_im) {
    // the library calls and allocations run without the GIL: other Python threads (the
    // harness's free-memory sampler, profiling.profile_op_gpu) keep running during a product
    pybind11::gil_scoped_release nogil;
    spg_handle_t h = reinterpret_cast<spg_handle_t>(handle);
    const spg_csr_t A = view(m, k, Ap, Aj, Ax), B = view(k, n, Bp, Bj, Bx);
    const spg_alg_t a = (spg_alg_t)alg;
    const float cf = (float)chunk_fraction;
    size_t ws_bytes = 0;
    spg_status_t st = spg_plan(h, &A, &B, a, cf, &ws_bytes, nullptr, nullptr);
    if (st) return {st, {}, {}, {}, 0, 0};
    const auto opt = Ax.options();
    at::Tensor ws = at::empty({(int64_t)std::max<size_t>(ws_bytes, 1)}, opt.dtype(at::kByte));
    // alpha as C's value type: one scalar, or (real, imag)
    double ad[2] = {alpha_re, alpha_im};
    float af[2] = {(float)alpha_re, (float)alpha_im};
    const void* alpha = (A.value_type == SPG_R_32F || A.value_type == SPG_C_32F) ? (const void*)af : (const void*)ad;
    int64_t nnz = 0;
    void *cj = nullptr, *cx = nullptr;
    size_t peak = 0;
    spg_plan_t plan = nullptr;
    at::Tensor indptr;
    // int64 row pointer once nnz(C) >= 2**31.  When the expected product count reaches 2**31
    // the first try is int64 already (an int32 try that overflows would redo the plan and
    // the symbolic pass); a result that fits is handed back with an int32 row pointer.
    const double avg_b = k > 0 ? (double)B.nnz / (double)k : 0.0;
    const bool wide = (double)A.nnz * avg_b >= 2147483648.0;
    for (at::ScalarType it : {wide ? at::kLong : at::kInt, at::kLong}) {
        indptr = at::empty({m + 1}, opt.dtype(it));
        st = spg_spgemm_ws(h, &A, &B, a, cf, alpha, ws.data_ptr(), ws_bytes, indptr.data_ptr(), itype(indptr), &nnz,
                           &cj, &cx, &peak, &plan);
        if (st != SPG_STATUS_OVERFLOW) break;
    }
    if (st) return {st, {}, {}, {}, 0, 0};
    const bool narrow = wide && nnz < 2147483648LL;   // back to the int32 contract
    at::Tensor indices, data;
    const int64_t vsz = Ax.element_size();
    if (cj) {   // ALG1: C sits compact (scaled) in the workspace
        const int64_t oj = (int64_t)((char*)cj - (char*)ws.data_ptr());
        const int64_t ox = (int64_t)((char*)cx - (char*)ws.data_ptr());
        indices = ws.slice(0, oj, oj + 4 * nnz).view(at::kInt);
        data = ws.slice(0, ox, ox + vsz * nnz).view(Ax.scalar_type());
    } else {
        indices = at::empty({nnz}, opt.dtype(at::kInt));
        data = at::empty({nnz}, opt);
        spg_csr_t C{m, n, nnz, indptr.data_ptr(), nnz ? indices.data_ptr() : nullptr, nnz ? data.data_ptr() : nullptr,
                    itype(indptr), A.value_type};
        st = spg_numeric(h, plan, alpha, &C);
        spg_plan_destroy(plan);
        if (st) return {st, {}, {}, {}, 0, 0};
    }
    if (narrow) indptr = indptr.to(at::kInt);   // stream-ordered after the numeric pass
    return {0, data, indices, indptr, (int64_t)ws_bytes, (int64_t)peak};
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, mod) {
    mod.def("spgemm", &spgemm, "plan + spg_spgemm_ws (+ spg_numeric) with torch allocations");
}
