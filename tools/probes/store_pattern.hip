// store_pattern.hip -- HBM write rate of the flow-entry expansion's store
// pattern (diagnostic).  4.68 GB (one 16.7 M-pair chunk of k=48 all-pairs
// entries) written three ways with 16-B stores:
//   fill   grid-stride, consecutive waves on consecutive 1-KB pieces;
//   group  wave w writes whole 17-KB groups g = w, w + nwaves, ... (the
//          expansion's order: ~8k groups written at once, 140 MB apart);
//   group+lds  the same with 4 LDS reads feeding every 16-B store.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probes/store_pattern tools/probes/store_pattern.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ __launch_bounds__(256) void fill_kernel(uint4 *o, size_t n16)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16;
         i += (size_t)gridDim.x * blockDim.x)
        o[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

template <bool LDS>
__global__ __launch_bounds__(256) void group_kernel(uint4 *o, size_t ngroups, int per_group16)
{
    __shared__ uint32_t buf[4][1024];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (LDS)
        for (int i = lane; i < 1024; i += 64) buf[wv][i] = i * 7u;
    __builtin_amdgcn_wave_barrier();
    const size_t nwaves = (size_t)gridDim.x * 4;
    for (size_t g = blockIdx.x * 4 + wv; g < ngroups; g += nwaves) {
        uint4 *p = o + g * per_group16;
        for (int t = lane; t < per_group16; t += 64) {
            uint4 v;
            if (LDS) {
                const int k = (t * 4) % 997;
                v = make_uint4(buf[wv][k], buf[wv][k + 1], buf[wv][k + 2], buf[wv][k + 3]);
            } else {
                v = make_uint4((uint32_t)t, 1u, 2u, (uint32_t)g);
            }
            p[t] = v;
        }
    }
}

int main()
{
    const size_t bytes = 4680ull << 20;
    const int per_group16 = 17 * 1024 / 16;            // 17-KB groups
    const size_t ngroups = bytes / (per_group16 * 16);
    uint4 *o;
    CK(hipMalloc(&o, bytes));
    CK(hipMemset(o, 0, bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    for (int rep = 0; rep < 3; ++rep) {
        for (int which = 0; which < 3; ++which) {
            CK(hipEventRecord(a));
            if (which == 0)
                hipLaunchKernelGGL(fill_kernel, dim3(cus * 8), dim3(256), 0, 0, o, bytes / 16);
            else if (which == 1)
                hipLaunchKernelGGL(group_kernel<false>, dim3(cus * 8), dim3(256), 0, 0, o, ngroups,
                                   per_group16);
            else
                hipLaunchKernelGGL(group_kernel<true>, dim3(cus * 8), dim3(256), 0, 0, o, ngroups,
                                   per_group16);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            const double wb = (which == 0 ? bytes : ngroups * per_group16 * 16.0);
            printf("%-10s %.3f ms  %.2f TB/s\n", which == 0 ? "fill" : which == 1 ? "group" : "group+lds",
                   ms, wb / (ms * 1e-3) / 1e12);
        }
    }
    return 0;
}
