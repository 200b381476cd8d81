// spgemm_from_txt.cpp -- native drivers spgemm_from_txt_alg{1,2,3} over libmi355_spgemm.so.
//
// Behavioural drop-in for the reference's cupy_cusparse/spgemm_from_txt_alg{1,2,3}.cu
// (main :104-208 / :117-242): same argv (`A_prefix B_prefix C_prefix [chunk_fraction]`),
// same CHUNK_FRACTION environment fallback and (0,1] check (alg3.cu:101-115), same text
// format (one value per line; indices %d; data parsed as double then narrowed to float,
// written with 9 significant digits; alg1.cu:19-78), same inference of A.cols = B.rows and
// B.cols = A.rows (alg1.cu:121-122), same validation (alg1.cu:80-102), same stdout line
// and exit codes (0 ok, 1 error, 2 usage).  The cuSPARSE generic-API sequence
// (alg1.cu:145-206) becomes spg_create / spg_plan x2 / spg_symbolic / spg_numeric.
//
// Built three times from this one source with -DSPG_DRIVER_ALG=1|2|3.  Deliberate
// differences: the ALG2 binary reports "ALG2" (the reference's alg2 prints "ALG3",
// spgemm_from_txt_alg2.cu:228); SPG_DTYPE=float64 runs the fp64 path (text is then
// written with 17 significant digits); the default stays fp32 like the reference.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "spgemm.h"

#ifndef SPG_DRIVER_ALG
#define SPG_DRIVER_ALG 1
#endif

#define CHECK_HIP(x)                                                                        \
    do {                                                                                    \
        hipError_t s_ = (x);                                                                \
        if (s_ != hipSuccess) {                                                             \
            std::fprintf(stderr, "HIP error %s:%d: %s\n", __FILE__, __LINE__,               \
                         hipGetErrorString(s_));                                            \
            std::exit(1);                                                                   \
        }                                                                                   \
    } while (0)
#define CHECK_SPG(x)                                                                        \
    do {                                                                                    \
        spg_status_t s_ = (x);                                                              \
        if (s_ != SPG_STATUS_SUCCESS) {                                                     \
            std::fprintf(stderr, "SpGEMM error %s:%d: %d (%s)\n", __FILE__, __LINE__,       \
                         (int)s_, spg_status_string(s_));                                   \
            std::exit(1);                                                                   \
        }                                                                                   \
    } while (0)

namespace {

// Whitespace-separated numbers, read in bulk (the reference uses ifstream >>).
bool slurp(const std::string& path, std::string& out) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) {
        std::perror(("open " + path).c_str());
        return false;
    }
    std::fseek(f, 0, SEEK_END);
    long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    out.resize(n > 0 ? (size_t)n : 0);
    size_t got = n > 0 ? std::fread(&out[0], 1, (size_t)n, f) : 0;
    std::fclose(f);
    out.resize(got);
    return true;
}

std::vector<int32_t> read_i32_list(const std::string& path) {
    std::string s;
    if (!slurp(path, s)) std::exit(1);
    std::vector<int32_t> v;
    v.reserve(s.size() / 4 + 1);
    const char* p = s.c_str();
    char* end = nullptr;
    for (;;) {
        long long x = std::strtoll(p, &end, 10);
        if (end == p) break;
        v.push_back((int32_t)x);
        p = end;
    }
    return v;
}

template <typename T>
std::vector<T> read_val_list(const std::string& path) {
    std::string s;
    if (!slurp(path, s)) std::exit(1);
    std::vector<T> v;
    v.reserve(s.size() / 8 + 1);
    const char* p = s.c_str();
    char* end = nullptr;
    for (;;) {
        double x = std::strtod(p, &end);
        if (end == p) break;
        v.push_back((T)x);
        p = end;
    }
    return v;
}

void write_i32_list(const std::string& path, const std::vector<int32_t>& v) {
    FILE* f = std::fopen(path.c_str(), "w");
    if (!f) { std::perror(("open " + path).c_str()); std::exit(1); }
    for (int32_t x : v) std::fprintf(f, "%d\n", x);
    std::fclose(f);
}

template <typename T>
void write_val_list(const std::string& path, const std::vector<T>& v) {
    FILE* f = std::fopen(path.c_str(), "w");
    if (!f) { std::perror(("open " + path).c_str()); std::exit(1); }
    const char* fmt = sizeof(T) == 4 ? "%.9g\n" : "%.17g\n";
    for (T x : v) std::fprintf(f, fmt, (double)x);
    std::fclose(f);
}

template <typename T>
struct CSR {
    int32_t rows{}, cols{-1}, nnz{};
    std::vector<int32_t> indptr, indices;
    std::vector<T> data;
};

template <typename T>
CSR<T> read_csr_txt_prefix(const std::string& prefix) {
    CSR<T> M;
    M.indptr = read_i32_list(prefix + "_indptr.txt");
    M.indices = read_i32_list(prefix + "_indices.txt");
    M.data = read_val_list<T>(prefix + "_data.txt");
    if (M.indptr.empty()) {
        std::fprintf(stderr, "empty indptr: %s\n", prefix.c_str());
        std::exit(1);
    }
    if (M.indices.size() != M.data.size()) {
        std::fprintf(stderr, "indices/data length mismatch for prefix %s\n", prefix.c_str());
        std::exit(1);
    }
    M.rows = (int32_t)M.indptr.size() - 1;
    M.nnz = (int32_t)M.indices.size();
    M.cols = -1;
    return M;
}

template <typename T>
void write_csr_txt_prefix(const std::string& prefix, const CSR<T>& M) {
    write_i32_list(prefix + "_indptr.txt", M.indptr);
    write_i32_list(prefix + "_indices.txt", M.indices);
    write_val_list<T>(prefix + "_data.txt", M.data);
}

template <typename T>
void validate_csr_indices(const CSR<T>& M, const char* name) {
    if (M.cols < 0) {
        std::fprintf(stderr, "[%s] cols not set before validation\n", name);
        std::exit(1);
    }
    if (!M.indices.empty()) {
        int32_t mx = *std::max_element(M.indices.begin(), M.indices.end());
        if (mx >= M.cols) {
            std::fprintf(stderr, "[%s] index out of bounds: max index %d >= ncols %d\n", name, mx,
                         M.cols);
            std::exit(1);
        }
        if (*std::min_element(M.indices.begin(), M.indices.end()) < 0) {
            std::fprintf(stderr, "[%s] negative column index detected\n", name);
            std::exit(1);
        }
    }
    if ((int)M.indptr.size() != M.rows + 1) {
        std::fprintf(stderr, "[%s] indptr length %zu != rows+1 (%d)\n", name, M.indptr.size(),
                     M.rows + 1);
        std::exit(1);
    }
}

float get_chunk_fraction(int argc, char** argv) {
    float cf = 0.2f;
    if (argc >= 5) {
        cf = std::strtof(argv[4], nullptr);
    } else {
        const char* s = std::getenv("CHUNK_FRACTION");
        if (s) cf = std::strtof(s, nullptr);
    }
    if (cf <= 0.0f || cf > 1.0f) {
        std::fprintf(stderr, "chunk_fraction must be in (0,1], got %f\n", cf);
        std::exit(1);
    }
    return cf;
}

template <typename T>
void* to_device(const std::vector<T>& v) {
    void* d = nullptr;
    CHECK_HIP(hipMalloc(&d, std::max<size_t>(v.size() * sizeof(T), 1)));
    if (!v.empty()) CHECK_HIP(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return d;
}

template <typename T>
int run(const std::string& Apre, const std::string& Bpre, const std::string& Cpre, float cf) {
    CSR<T> A = read_csr_txt_prefix<T>(Apre);
    CSR<T> B = read_csr_txt_prefix<T>(Bpre);
    if (A.rows <= 0 || B.rows <= 0) {
        std::fprintf(stderr, "invalid rows: A.rows=%d B.rows=%d\n", A.rows, B.rows);
        return 1;
    }
    A.cols = B.rows;
    B.cols = A.rows;
    validate_csr_indices(A, "A");
    validate_csr_indices(B, "B");

    const spg_dtype_t vt = sizeof(T) == 8 ? SPG_R_64F : SPG_R_32F;
    spg_csr_t dA{A.rows, A.cols, A.nnz, to_device(A.indptr), to_device(A.indices), to_device(A.data),
                 SPG_INDEX_32I, vt};
    spg_csr_t dB{B.rows, B.cols, B.nnz, to_device(B.indptr), to_device(B.indices), to_device(B.data),
                 SPG_INDEX_32I, vt};

    spg_handle_t h;
    CHECK_SPG(spg_create(&h, -1));
    const spg_alg_t alg = (spg_alg_t)SPG_DRIVER_ALG;

    size_t ws_bytes = 0;
    CHECK_SPG(spg_plan(h, &dA, &dB, alg, cf, &ws_bytes, nullptr, nullptr));
    void* ws = nullptr;
    CHECK_HIP(hipMalloc(&ws, std::max<size_t>(ws_bytes, 1)));
    spg_plan_t plan;
    CHECK_SPG(spg_plan(h, &dA, &dB, alg, cf, &ws_bytes, ws, &plan));

    int64_t num_prods = 0;
    CHECK_SPG(spg_num_products(h, plan, &num_prods));
    (void)num_prods;

    int32_t* dCptr = nullptr;
    CHECK_HIP(hipMalloc((void**)&dCptr, (A.rows + 1) * sizeof(int32_t)));
    int64_t Cnnz = 0;
    CHECK_SPG(spg_symbolic(h, plan, dCptr, SPG_INDEX_32I, &Cnnz));
    void *dCind = nullptr, *dCval = nullptr;
    CHECK_HIP(hipMalloc(&dCind, std::max<size_t>((size_t)Cnnz * sizeof(int32_t), 1)));
    CHECK_HIP(hipMalloc(&dCval, std::max<size_t>((size_t)Cnnz * sizeof(T), 1)));
    spg_csr_t dC{A.rows, B.cols, Cnnz, dCptr, dCind, dCval, SPG_INDEX_32I, vt};
    const T alpha = (T)1;
    CHECK_SPG(spg_numeric(h, plan, &alpha, &dC));

    CSR<T> C;
    C.rows = A.rows;
    C.cols = B.cols;
    C.nnz = (int32_t)Cnnz;
    C.indptr.resize(C.rows + 1);
    C.indices.resize(C.nnz);
    C.data.resize(C.nnz);
    CHECK_HIP(hipMemcpy(C.indptr.data(), dCptr, (C.rows + 1) * sizeof(int32_t), hipMemcpyDeviceToHost));
    if (C.nnz) {
        CHECK_HIP(hipMemcpy(C.indices.data(), dCind, C.nnz * sizeof(int32_t), hipMemcpyDeviceToHost));
        CHECK_HIP(hipMemcpy(C.data.data(), dCval, C.nnz * sizeof(T), hipMemcpyDeviceToHost));
    }
    write_csr_txt_prefix(Cpre, C);
    std::printf("[C++] ALG%d wrote %s_* (rows=%d, cols=%d, nnz=%d", SPG_DRIVER_ALG, Cpre.c_str(),
                C.rows, C.cols, C.nnz);
    if (SPG_DRIVER_ALG != 1) std::printf(", chunk_fraction=%g", (double)cf);
    std::printf(")\n");

    CHECK_SPG(spg_plan_destroy(plan));
    CHECK_SPG(spg_destroy(h));
    for (void* p : {dA.indptr, dA.indices, dA.values, dB.indptr, dB.indices, dB.values,
                    (void*)dCptr, dCind, dCval, ws})
        (void)hipFree(p);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) {
        if (SPG_DRIVER_ALG == 1)
            std::fprintf(stderr, "Usage: %s A_prefix B_prefix C_prefix\n", argv[0]);
        else
            std::fprintf(stderr, "Usage: %s A_prefix B_prefix C_prefix [chunk_fraction]\n", argv[0]);
        return 2;
    }
    const std::string Apre = argv[1], Bpre = argv[2], Cpre = argv[3];
    const float cf = SPG_DRIVER_ALG == 1 ? 0.2f : get_chunk_fraction(argc, argv);
    const char* dt = std::getenv("SPG_DTYPE");
    if (dt && std::strcmp(dt, "float64") == 0) return run<double>(Apre, Bpre, Cpre, cf);
    return run<float>(Apre, Bpre, Cpre, cf);
}
