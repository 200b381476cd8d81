// abtest/gather_probe.hip -- memory-system probe for the tile kernels' access shape, and the
// calibration of the TCC byte counters for it (VERDICT r03 "make the traffic figure evidence").
//
//   stream  S_MB                 every lane reads 16 B per load (dwordx4), the whole buffer once:
//                                the known-bytes case FETCH_SIZE's x2 rule was measured on
//   gather  S_MB L [store]       12-byte records (value f64 + column u32, the tile-major B record)
//                                gathered as the flattened (jj, kk) walk does it: segments of L
//                                consecutive records at random record positions inside a slice of
//                                S_MB per XCD group (blocks b and b+8 share a slice, as the tile
//                                kernels' XCD-aware item map gives every XCD its own tile), 64
//                                products per wave instruction, 8 instructions in flight; with
//                                `store` also a non-temporal 12-byte-per-2-products output stream
//                                (C's columns and values)
//
// Prints one JSON line per run: useful bytes (12 per product, + the stream), kernel ms, GB/s.
// Under `rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
// TCC_EA0_RDREQ_sum` the request mix gives the fabric bytes exactly (32/64/128-B requests).
// Build: hipcc -O3 --offload-arch=gfx950 abtest/gather_probe.hip -o abtest/gather_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(2);                                                            \
        }                                                                            \
    } while (0)

constexpr int WPB = 2;   // waves per block, as k_tile_dn

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__global__ __launch_bounds__(256) void k_stream(const uint4* __restrict__ p, int64_t n, unsigned* sink) {
    uint32_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// One wave: `chunks` wave instructions of 64 products, U in flight.  Product t of the wave
// belongs to segment t / L at a random start inside the group's slice.  RB = record bytes (12:
// value + column as one dwordx3; 16: padded to one dwordx4).
template <int U, int RB>
__global__ __launch_bounds__(WPB * 64) void k_gather(const uint32_t* __restrict__ rec, int64_t slice_recs, int L,
                                                     int chunks, int store, int32_t* __restrict__ cj,
                                                     double* __restrict__ cx, int64_t out_per_wave,
                                                     double* sink, int align) {
    const int l = threadIdx.x & 63;
    const uint32_t wave = blockIdx.x * WPB + (threadIdx.x >> 6);
    const int64_t base = (int64_t)(blockIdx.x & 7) * slice_recs;
    const uint32_t span = (uint32_t)(slice_recs - L);
    const char* rb = reinterpret_cast<const char*>(rec) + base * RB;
    double acc = 0.0;
    int32_t* cjw = cj + (int64_t)wave * out_per_wave;
    double* cxw = cx + (int64_t)wave * out_per_wave;
    int64_t op = 0;
    for (int c0 = 0; c0 < chunks; c0 += U) {
        double v[U];
        int col[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t t = (uint32_t)(c0 + u) * 64u + (uint32_t)l;
            const uint32_t seg = t / (uint32_t)L, kk = t - seg * (uint32_t)L;
            const uint32_t r = mix(seg * 2654435761u ^ wave * 40503u);
            // align: every segment starts at a 128-byte line (the slice holds slice_recs*RB/128 lines)
            const uint64_t sb = align ? (uint64_t)(r % (uint32_t)((slice_recs * RB) / 128 - 2)) * 128u
                                      : (uint64_t)(r % span) * RB;
            if constexpr (RB == 12) {
                const uint3 x = *reinterpret_cast<const uint3*>(rb + sb + (uint64_t)kk * 12u);
                v[u] = __hiloint2double((int)x.y, (int)x.x);
                col[u] = (int)x.z;
            } else {
                const uint4 x = *reinterpret_cast<const uint4*>(rb + sb + (uint64_t)kk * 16u);
                v[u] = __hiloint2double((int)x.y, (int)x.x);
                col[u] = (int)x.z;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            acc += v[u];
            if (store && (u & 1) == 0 && op + 64 <= out_per_wave) {
                __builtin_nontemporal_store(col[u], cjw + op + l);
                __builtin_nontemporal_store(v[u], cxw + op + l);
                op += 64;
            }
        }
    }
    if (acc == 123.456) sink[0] = acc;
}

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: gather_probe stream S_MB | gather S_MB L [store] [waves_per_cu] [U] [rec_bytes]\n");
        return 1;
    }
    const bool stream = std::strcmp(argv[1], "stream") == 0;
    const double smb = std::atof(argv[2]);
    double* sink;
    CK(hipMalloc(&sink, 64));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    if (stream) {
        const int64_t bytes = (int64_t)(smb * 1048576.0) / 16 * 16;
        uint4* p;
        CK(hipMalloc(&p, bytes));
        CK(hipMemset(p, 1, bytes));
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(k_stream, dim3(2048), dim3(256), 0, 0, p, bytes / 16, (unsigned*)sink);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (ms < best) best = ms;
        }
        std::printf("{\"mode\": \"stream\", \"bytes_per_launch\": %lld, \"launches\": 5, \"best_ms\": %.4f, \"GBps\": %.1f}\n",
                    (long long)bytes, best, bytes / (best * 1e-3) / 1e9);
        return 0;
    }
    const int L = argc > 3 ? std::atoi(argv[3]) : 10;
    const int store = argc > 4 ? std::atoi(argv[4]) : 0;
    const int wpc = argc > 5 ? std::atoi(argv[5]) : 8;       // waves per CU (one generation)
    const int U = argc > 6 ? std::atoi(argv[6]) : 8;         // loads in flight per wave (8 or 16)
    const int RB = argc > 7 ? std::atoi(argv[7]) : 12;       // record bytes (12 or 16)
    const int align = argc > 8 ? std::atoi(argv[8]) : 0;      // segments start at 128-byte lines
    const int64_t total_chunks = (int64_t)256 * 32 * 4096;   // 2^25 wave instructions = 2^31 products
    const int chunks = (int)(total_chunks / (256 * wpc));
    const int64_t slice = (int64_t)(smb * 1048576.0) / RB;
    const int64_t total = 8 * slice;
    uint32_t* rec;
    CK(hipMalloc(&rec, total * RB + 256));
    {
        std::vector<uint32_t> h((size_t)total * RB / 4);
        for (int64_t i = 0; i < (int64_t)h.size() / 4; ++i) {
            const double v = 1.0 + (double)(i % 1000) * 1e-3;
            std::memcpy(&h[(size_t)i * 4], &v, 8);
            h[(size_t)i * 4 + 2] = (uint32_t)(i & 2047);
        }
        CK(hipMemcpy(rec, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    }
    const int blocks = 256 * wpc / WPB;
    const int waves = blocks * WPB;
    const int64_t out_per_wave = store ? (int64_t)(chunks / 2) * 64 : 0;
    int32_t* cj = nullptr;
    double* cx = nullptr;
    if (store) {
        CK(hipMalloc(&cj, (size_t)waves * out_per_wave * 4));
        CK(hipMalloc(&cx, (size_t)waves * out_per_wave * 8));
    }
    float best = 1e30f;
    const int reps = 5;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a));
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(WPB * 64), 0, 0, rec, slice, L, chunks, store, cj, cx,
                               out_per_wave, sink, align);
        };
        if (U == 16) { if (RB == 16) go(k_gather<16, 16>); else go(k_gather<16, 12>); }
        else { if (RB == 16) go(k_gather<8, 16>); else go(k_gather<8, 12>); }
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipGetLastError());
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    const double products = (double)waves * chunks * 64;
    const double rbytes = (double)RB * products;
    const double wbytes = store ? 12.0 * (double)waves * out_per_wave : 0.0;
    std::printf("{\"mode\": \"gather\", \"slice_MB\": %.2f, \"L\": %d, \"store\": %d, \"waves_per_cu\": %d, \"U\": %d, \"rec_bytes\": %d, \"align\": %d, \"launches\": %d, "
                "\"products\": %.0f, \"record_bytes_per_launch\": %.0f, \"store_bytes_per_launch\": %.0f, "
                "\"best_ms\": %.4f, \"record_GBps\": %.1f, \"total_GBps\": %.1f}\n",
                smb, L, store, wpc, U, RB, align, reps, products, rbytes, wbytes, best, rbytes / (best * 1e-3) / 1e9,
                (rbytes + wbytes) / (best * 1e-3) / 1e9);
    return 0;
}
