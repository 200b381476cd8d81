// abtest/lds_fadd_order.hip -- hardware check behind the tile kernel's ordered accumulation.
//
// Questions (answered on the GPU box; the shipped kernels rely on none of this unless the
// answers are "yes" on every trial):
//   Q1  ds_add_f64 (LDS atomic add, no return) rounds exactly like v_add_f64: IEEE
//       round-to-nearest-even, denormals kept, -0, inf and nan as v_add_f64.
//   Q2  lanes of ONE wave instruction that hit the same LDS address are applied in
//       ascending lane order (so the earlier product of a 64-product chunk adds first).
//   Q3  the same for ds_add_rtn_f64 (the returned old values show the order directly).
// Build: hipcc -O3 --offload-arch=gfx950 abtest/lds_fadd_order.hip -o abtest/lds_fadd_order
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return 2;                                                                \
        }                                                                            \
    } while (0)

constexpr int SLOTS = 1024;

// Q2/Q3: block of 64 lanes (one wave); trial t: lane l adds v[t*64+l] at slot a[t*64+l] if
// act bit l is set; slots start at init[t*SLOTS + s]. out = final slots; ret = returned old
// value of each lane (rtn variant).
template <bool RTN>
__global__ __launch_bounds__(64) void k_order(int trials, const double* __restrict__ init, const double* __restrict__ v,
                                              const int* __restrict__ a, const unsigned long long* __restrict__ act,
                                              double* __restrict__ out, double* __restrict__ ret) {
    __shared__ double s[SLOTS];
    const int l = threadIdx.x;
    for (int t = blockIdx.x; t < trials; t += gridDim.x) {
        for (int i = l; i < SLOTS; i += 64) s[i] = init[(size_t)t * SLOTS + i];
        __syncthreads();
        const double x = v[(size_t)t * 64 + l];
        const int ad = a[(size_t)t * 64 + l];
        if ((act[t] >> l) & 1ull) {
            if constexpr (RTN) {
                ret[(size_t)t * 64 + l] = __hip_atomic_fetch_add(&s[ad], x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else {
                __hip_atomic_fetch_add(&s[ad], x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        __syncthreads();
        for (int i = l; i < SLOTS; i += 64) out[(size_t)t * SLOTS + i] = s[i];
        __syncthreads();
    }
}

// Q1: lane-private slots: s[l] = x; ds_add_f64 s[l] += y; compare with v_add_f64 x + y.
__global__ __launch_bounds__(64) void k_round(int n, const double* __restrict__ x, const double* __restrict__ y,
                                              double* __restrict__ lds_sum, double* __restrict__ valu_sum) {
    __shared__ double s[64];
    const int l = threadIdx.x;
    for (int i = blockIdx.x * 64 + l; i < n; i += gridDim.x * 64) {
        s[l] = x[i];
        __hip_atomic_fetch_add(&s[l], y[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        lds_sum[i] = s[l];
        valu_sum[i] = __dadd_rn(x[i], y[i]);
    }
}

// Q4/Q5: the same two questions for ds_add_f32 (LDS atomic float add).
__global__ __launch_bounds__(64) void k_round32(int n, const float* __restrict__ x, const float* __restrict__ y,
                                                float* __restrict__ lds_sum, float* __restrict__ valu_sum) {
    __shared__ float s[64];
    const int l = threadIdx.x;
    for (int i = blockIdx.x * 64 + l; i < n; i += gridDim.x * 64) {
        s[l] = x[i];
        __hip_atomic_fetch_add(&s[l], y[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        lds_sum[i] = s[l];
        valu_sum[i] = __fadd_rn(x[i], y[i]);
    }
}
__global__ __launch_bounds__(64) void k_order32(int trials, const float* __restrict__ init, const float* __restrict__ v,
                                                const int* __restrict__ a, const unsigned long long* __restrict__ act,
                                                float* __restrict__ out) {
    __shared__ float s[SLOTS];
    const int l = threadIdx.x;
    for (int t = blockIdx.x; t < trials; t += gridDim.x) {
        for (int i = l; i < SLOTS; i += 64) s[i] = init[(size_t)t * SLOTS + i];
        __syncthreads();
        if ((act[t] >> l) & 1ull)
            __hip_atomic_fetch_add(&s[a[(size_t)t * 64 + l]], v[(size_t)t * 64 + l], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __syncthreads();
        for (int i = l; i < SLOTS; i += 64) out[(size_t)t * SLOTS + i] = s[i];
        __syncthreads();
    }
}

static bool same_bits32(float a, float b) {
    if (std::isnan(a) && std::isnan(b)) return true;
    uint32_t x, y;
    std::memcpy(&x, &a, 4);
    std::memcpy(&y, &b, 4);
    return x == y;
}

static bool same_bits(double a, double b) {
    if (std::isnan(a) && std::isnan(b)) return true;
    uint64_t x, y;
    std::memcpy(&x, &a, 8);
    std::memcpy(&y, &b, 8);
    return x == y;
}

static double rnd_value(std::mt19937_64& g, int mode) {
    std::uniform_real_distribution<double> u(1.0, 2.0);
    std::uniform_int_distribution<int> e(-60, 60), sgn(0, 1);
    double m = u(g) * (sgn(g) ? -1.0 : 1.0);
    switch (mode) {
        case 0: return std::ldexp(m, e(g));                       // wide exponents: order shows
        case 1: return std::ldexp(m, std::uniform_int_distribution<int>(-1074, -1000)(g));   // denormal range
        case 2: return std::ldexp(m, std::uniform_int_distribution<int>(-3, 3)(g));   // close magnitudes
        default: {
            const double sp[] = {INFINITY, -INFINITY, NAN, 0.0, -0.0, 4.9e-324, -4.9e-324, 1.7976931348623157e308};
            return sp[std::uniform_int_distribution<int>(0, 7)(g)];
        }
    }
}

int main(int argc, char** argv) {
    const int trials = argc > 1 ? std::atoi(argv[1]) : 50000;
    std::mt19937_64 g(12345);
    // ---- Q1
    const int n1 = 1 << 22;
    std::vector<double> x(n1), y(n1), ls(n1), vs(n1);
    for (int i = 0; i < n1; ++i) {
        const int mode = (i >> 18) & 3;
        x[i] = rnd_value(g, mode);
        y[i] = rnd_value(g, (mode + (i & 1)) & 3);
        if ((i & 7) == 3) y[i] = -x[i] * (1.0 + std::ldexp(1.0, -52));   // near-cancellation
    }
    double *dx, *dy, *dl, *dv;
    CK(hipMalloc(&dx, 8 * n1)); CK(hipMalloc(&dy, 8 * n1)); CK(hipMalloc(&dl, 8 * n1)); CK(hipMalloc(&dv, 8 * n1));
    CK(hipMemcpy(dx, x.data(), 8 * n1, hipMemcpyHostToDevice));
    CK(hipMemcpy(dy, y.data(), 8 * n1, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_round, dim3(4096), dim3(64), 0, 0, n1, dx, dy, dl, dv);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(ls.data(), dl, 8 * n1, hipMemcpyDeviceToHost));
    CK(hipMemcpy(vs.data(), dv, 8 * n1, hipMemcpyDeviceToHost));
    long bad1 = 0, badc = 0;
    for (int i = 0; i < n1; ++i) {
        if (!same_bits(ls[i], vs[i])) { if (bad1 < 5) std::printf("Q1 mismatch x=%a y=%a lds=%a valu=%a\n", x[i], y[i], ls[i], vs[i]); ++bad1; }
        if (!same_bits(vs[i], x[i] + y[i])) ++badc;
    }
    std::printf("Q1 ds_add_f64 vs v_add_f64: %d cases, %ld mismatches (v_add_f64 vs host: %ld)\n", n1, bad1, badc);

    // ---- Q2 / Q3
    std::vector<double> init((size_t)trials * SLOTS, 0.0), v((size_t)trials * 64), out((size_t)trials * SLOTS), ret((size_t)trials * 64);
    std::vector<int> a((size_t)trials * 64);
    std::vector<unsigned long long> act(trials);
    for (int t = 0; t < trials; ++t) {
        const int pat = t % 5;
        const int range = pat == 0 ? 1 : pat == 1 ? 4 : pat == 2 ? 64 : pat == 3 ? 1024 : 16;
        for (int l = 0; l < 64; ++l) {
            a[(size_t)t * 64 + l] = std::uniform_int_distribution<int>(0, range - 1)(g) * (pat == 4 ? 64 : 1);   // pat 4: one bank
            v[(size_t)t * 64 + l] = rnd_value(g, (t / 5) % 3);
        }
        act[t] = (t & 1) ? g() : ~0ull;
        for (int s = 0; s < range; ++s) init[(size_t)t * SLOTS + s * (pat == 4 ? 64 : 1)] = rnd_value(g, 2);
    }
    double *di, *dv2, *dout, *dret;
    int* da;
    unsigned long long* dact;
    CK(hipMalloc(&di, 8 * init.size())); CK(hipMalloc(&dv2, 8 * v.size())); CK(hipMalloc(&dout, 8 * out.size()));
    CK(hipMalloc(&dret, 8 * ret.size())); CK(hipMalloc(&da, 4 * a.size())); CK(hipMalloc(&dact, 8 * act.size()));
    CK(hipMemcpy(di, init.data(), 8 * init.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dv2, v.data(), 8 * v.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(da, a.data(), 4 * a.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dact, act.data(), 8 * act.size(), hipMemcpyHostToDevice));
    for (int rtn = 0; rtn < 2; ++rtn) {
        if (rtn) hipLaunchKernelGGL(k_order<true>, dim3(2048), dim3(64), 0, 0, trials, di, dv2, da, dact, dout, dret);
        else hipLaunchKernelGGL(k_order<false>, dim3(2048), dim3(64), 0, 0, trials, di, dv2, da, dact, dout, dret);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(out.data(), dout, 8 * out.size(), hipMemcpyDeviceToHost));
        CK(hipMemcpy(ret.data(), dret, 8 * ret.size(), hipMemcpyDeviceToHost));
        long bad = 0, badrev = 0, badret = 0, conflicts = 0;
        for (int t = 0; t < trials; ++t) {
            std::vector<double> s(init.begin() + (size_t)t * SLOTS, init.begin() + (size_t)(t + 1) * SLOTS), r = s;
            std::vector<int> hits(SLOTS, 0);
            bool ok = true, okr = true, okret = true;
            for (int l = 0; l < 64; ++l) {
                if (!((act[t] >> l) & 1ull)) continue;
                const int ad = a[(size_t)t * 64 + l];
                if (hits[ad]++) ++conflicts;
                const double old = s[ad];
                s[ad] = s[ad] + v[(size_t)t * 64 + l];
                if (rtn && !same_bits(ret[(size_t)t * 64 + l], old)) okret = false;
            }
            for (int l = 63; l >= 0; --l)
                if ((act[t] >> l) & 1ull) r[a[(size_t)t * 64 + l]] += v[(size_t)t * 64 + l];
            for (int i = 0; i < SLOTS; ++i) {
                if (!same_bits(out[(size_t)t * SLOTS + i], s[i])) ok = false;
                if (!same_bits(out[(size_t)t * SLOTS + i], r[i])) okr = false;
            }
            if (!ok) ++bad;
            if (!okr) ++badrev;
            if (!okret) ++badret;
        }
        std::printf("Q%d %s: %d trials, %ld same-address lane pairs; mismatches vs ascending-lane order %ld, "
                    "vs descending %ld%s\n", rtn ? 3 : 2, rtn ? "ds_add_rtn_f64" : "ds_add_f64", trials, conflicts,
                    bad, badrev, rtn ? (badret ? " (returned old values out of order)" : " (returned old values in lane order)") : "");
    }
    // ---- Q4 (f32 rounding incl. denormals) and Q5 (f32 lane order)
    {
        std::vector<float> xf(n1), yf(n1), lf(n1), vf(n1);
        for (int i = 0; i < n1; ++i) {
            const int mode = (i >> 18) & 3;
            auto rv = [&](int m) -> float {
                std::uniform_real_distribution<float> u(1.0f, 2.0f);
                const float mm = u(g) * ((g() & 1) ? -1.f : 1.f);
                if (m == 0) return std::ldexp(mm, std::uniform_int_distribution<int>(-30, 30)(g));
                if (m == 1) return std::ldexp(mm, std::uniform_int_distribution<int>(-149, -120)(g));   // denormals
                if (m == 2) return std::ldexp(mm, std::uniform_int_distribution<int>(-3, 3)(g));
                const float sp[] = {INFINITY, -INFINITY, NAN, 0.0f, -0.0f, 1.4e-45f, -1.4e-45f, 3.4028235e38f};
                return sp[std::uniform_int_distribution<int>(0, 7)(g)];
            };
            xf[i] = rv(mode);
            yf[i] = rv((mode + (i & 1)) & 3);
        }
        float *dxf, *dyf, *dlf, *dvf;
        CK(hipMalloc(&dxf, 4 * n1)); CK(hipMalloc(&dyf, 4 * n1)); CK(hipMalloc(&dlf, 4 * n1)); CK(hipMalloc(&dvf, 4 * n1));
        CK(hipMemcpy(dxf, xf.data(), 4 * n1, hipMemcpyHostToDevice));
        CK(hipMemcpy(dyf, yf.data(), 4 * n1, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_round32, dim3(4096), dim3(64), 0, 0, n1, dxf, dyf, dlf, dvf);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(lf.data(), dlf, 4 * n1, hipMemcpyDeviceToHost));
        CK(hipMemcpy(vf.data(), dvf, 4 * n1, hipMemcpyDeviceToHost));
        long b4 = 0, b4h = 0;
        for (int i = 0; i < n1; ++i) {
            if (!same_bits32(lf[i], vf[i])) { if (b4 < 5) std::printf("Q4 mismatch x=%a y=%a lds=%a valu=%a\n", xf[i], yf[i], lf[i], vf[i]); ++b4; }
            if (!same_bits32(vf[i], xf[i] + yf[i])) ++b4h;
        }
        std::printf("Q4 ds_add_f32 vs v_add_f32: %d cases, %ld mismatches (v_add_f32 vs host: %ld)\n", n1, b4, b4h);
        std::vector<float> initf((size_t)trials * SLOTS), vv((size_t)trials * 64), outf((size_t)trials * SLOTS);
        for (size_t i = 0; i < initf.size(); ++i) initf[i] = (float)init[i];
        for (size_t i = 0; i < vv.size(); ++i) vv[i] = (float)v[i];
        float *di2, *dv3, *do2;
        CK(hipMalloc(&di2, 4 * initf.size())); CK(hipMalloc(&dv3, 4 * vv.size())); CK(hipMalloc(&do2, 4 * outf.size()));
        CK(hipMemcpy(di2, initf.data(), 4 * initf.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(dv3, vv.data(), 4 * vv.size(), hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_order32, dim3(2048), dim3(64), 0, 0, trials, di2, dv3, da, dact, do2);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(outf.data(), do2, 4 * outf.size(), hipMemcpyDeviceToHost));
        long bad = 0, badrev = 0;
        for (int t = 0; t < trials; ++t) {
            std::vector<float> s(initf.begin() + (size_t)t * SLOTS, initf.begin() + (size_t)(t + 1) * SLOTS), r = s;
            for (int l = 0; l < 64; ++l)
                if ((act[t] >> l) & 1ull) s[a[(size_t)t * 64 + l]] = s[a[(size_t)t * 64 + l]] + vv[(size_t)t * 64 + l];
            for (int l = 63; l >= 0; --l)
                if ((act[t] >> l) & 1ull) r[a[(size_t)t * 64 + l]] += vv[(size_t)t * 64 + l];
            bool ok = true, okr = true;
            for (int i = 0; i < SLOTS; ++i) {
                if (!same_bits32(outf[(size_t)t * SLOTS + i], s[i])) ok = false;
                if (!same_bits32(outf[(size_t)t * SLOTS + i], r[i])) okr = false;
            }
            bad += !ok;
            badrev += !okr;
        }
        std::printf("Q5 ds_add_f32: %d trials; mismatches vs ascending-lane order %ld, vs descending %ld\n", trials, bad, badrev);
    }
    return 0;
}
