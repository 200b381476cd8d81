// Device check of the wave-level primitives in spg_device.hpp (DPP scans).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "spg_device.hpp"
using namespace spg;
__global__ void k(const int* in, int* sum_out, int* max_out) {
    const int l = lane_id();
    const int v = in[blockIdx.x * 64 + l];
    sum_out[blockIdx.x * 64 + l] = wave_incl_sum_dpp(v);
    max_out[blockIdx.x * 64 + l] = wave_incl_max_dpp(v);
}
int main() {
    const int nb = 64, n = nb * 64;
    int *h = (int*)malloc(n * 4), *hs = (int*)malloc(n * 4), *hm = (int*)malloc(n * 4);
    srand(1);
    for (int i = 0; i < n; ++i) h[i] = (rand() % 9) - 1;   // values >= -1
    int *d, *ds, *dm;
    hipMalloc(&d, n * 4); hipMalloc(&ds, n * 4); hipMalloc(&dm, n * 4);
    hipMemcpy(d, h, n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(nb), dim3(64), 0, 0, d, ds, dm);
    hipMemcpy(hs, ds, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(hm, dm, n * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int b = 0; b < nb; ++b) {
        int s = 0, m = -1;
        for (int l = 0; l < 64; ++l) {
            s += h[b * 64 + l];
            m = h[b * 64 + l] > m ? h[b * 64 + l] : m;
            if (hs[b * 64 + l] != s || hm[b * 64 + l] != m) {
                if (bad < 10) printf("block %d lane %d: sum %d want %d, max %d want %d\n", b, l, hs[b*64+l], s, hm[b*64+l], m);
                ++bad;
            }
        }
    }
    printf("wave_scan_check: %s (%d bad)\n", bad ? "FAIL" : "OK", bad);
    return bad ? 1 : 0;
}
