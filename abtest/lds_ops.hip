// abtest/lds_ops.hip -- throughput of the LDS operations an ordered accumulation can use,
// at random addresses inside one wave's 1024-slot accumulator (the dense tile's shape), with
// 14 waves per CU.  Prints cycles per wave-instruction per CU for each op.
// Build: hipcc -O3 --offload-arch=gfx950 abtest/lds_ops.hip -o abtest/lds_ops
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int SLOTS = 1024;
constexpr int WPB = 2;
constexpr int ITERS = 4096;

template <int OP>
__global__ __launch_bounds__(WPB * 64) void k_ops(unsigned seed, double* sink) {
    __shared__ double acc[WPB][SLOTS + 64];
    __shared__ unsigned char hit[WPB][SLOTS + 64];
    __shared__ unsigned bits[WPB][SLOTS / 32];
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = l; i < SLOTS; i += 64) { acc[w][i] = 0.0; hit[w][i] = 0; }
    if (l < SLOTS / 32) bits[w][l] = 0;
    __syncthreads();
    unsigned x = seed ^ (blockIdx.x * 7919u) ^ (l * 104729u);
    double v = 1.0 + l;
    double r = 0.0;
    for (int it = 0; it < ITERS; ++it) {
        x = x * 1664525u + 1013904223u;
        const int c = (x >> 8) & (SLOTS - 1);
        if constexpr (OP == 0) {
            __hip_atomic_fetch_add(&acc[w][c], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if constexpr (OP == 1) {
            hit[w][c] = 1;
        } else if constexpr (OP == 2) {
            __hip_atomic_fetch_add(&acc[w][c], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            hit[w][c] = 1;
        } else if constexpr (OP == 3) {
            acc[w][c] = acc[w][c] + v;   // read-add-write (not ordered across lanes)
        } else if constexpr (OP == 4) {
            atomicOr(&bits[w][c >> 5], 1u << (c & 31));
        } else if constexpr (OP == 5) {
            r += acc[w][c];
        } else if constexpr (OP == 6) {
            __hip_atomic_fetch_add(&acc[w][c], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            atomicOr(&bits[w][c >> 5], 1u << (c & 31));
        } else if constexpr (OP == 7) {
            // two f32 halves of the column's slot (a u32 atomic add stands in for the pair)
            atomicAdd(reinterpret_cast<unsigned*>(&acc[w][0]) + 2 * c, 1u);
        } else if constexpr (OP == 8) {
            __hip_atomic_fetch_add(reinterpret_cast<float*>(&acc[w][0]) + c, (float)v, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if constexpr (OP == 9) {
            __hip_atomic_fetch_add(reinterpret_cast<float*>(&acc[w][0]) + 2 * c, (float)v, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    __syncthreads();
    double s = r;
    for (int i = l; i < SLOTS; i += 64) s += acc[w][i] + hit[w][i];
    if (l < SLOTS / 32) s += bits[w][l];
    if (s == 123.456) sink[0] = s;
}

template <int OP>
float run(int blocks, double* sink) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(k_ops<OP>, dim3(blocks), dim3(WPB * 64), 0, 0, 1u, sink);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k_ops<OP>, dim3(blocks), dim3(WPB * 64), 0, 0, 2u, sink);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const int blocks = cus * 7;   // 14 waves per CU
    double* sink;
    (void)hipMalloc(&sink, 8);
    const double clk = p.clockRate * 1e3;   // Hz
    const char* names[] = {"ds_add_f64", "ds_write_b8 (hit)", "ds_add_f64 + ds_write_b8", "ds_read_b64+add+ds_write_b64",
                           "ds_or_b32 (bitmap)", "ds_read_b64", "ds_add_f64 + ds_or_b32", "ds_add_u32", "ds_add_f32 (dense slots)",
                           "ds_add_f32 (stride-2 slots)"};
    float t[10] = {run<0>(blocks, sink), run<1>(blocks, sink), run<2>(blocks, sink), run<3>(blocks, sink),
                   run<4>(blocks, sink), run<5>(blocks, sink), run<6>(blocks, sink), run<7>(blocks, sink),
                   run<8>(blocks, sink), run<9>(blocks, sink)};
    const double waves_per_cu = (double)blocks * WPB / cus;
    for (int i = 0; i < 10; ++i) {
        const double cyc = t[i] * 1e-3 * clk;   // cycles of the run
        std::printf("%-32s %8.3f ms  %6.2f CU-cycles per wave-instruction\n", names[i], t[i],
                    cyc / (waves_per_cu * ITERS));
    }
    return 0;
}
