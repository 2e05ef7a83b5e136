// simd_probe.hip -- where the waves of a workgroup land (diagnostic).
//
// dfs_async_kernel gives wave 0 of every workgroup the search and waves
// 1..NW-1 the decrements.  If the dispatcher puts wave w of each workgroup on
// SIMD w of its CU, the 4-5 co-resident search waves of a CU share one SIMD's
// issue while the workers spread over the other three.  This launches the
// headline's shape (1,152 workgroups of NW waves, the same LDS per
// workgroup), keeps every wave resident for a while, and records each wave's
// HW_ID (CU, SIMD) and XCC_ID; the host prints, per CU, how many wave-0s
// share a SIMD.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/simd_probe tools/simd_probe.hip
// Run:   tools/simd_probe [workgroups=1152] [waves=4] [lds_bytes=31792]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

// s_getreg encodings: (size - 1) << 11 | offset << 6 | register id
constexpr int kHwId = (31 << 11) | 4;     // HW_REG_HW_ID, all 32 bits
constexpr int kXccId = (15 << 11) | 20;   // HW_REG_XCC_ID, low 16 bits

__global__ void probe(uint32_t *out, int spins)
{
    extern __shared__ uint32_t lds[];
    const uint32_t hw = __builtin_amdgcn_s_getreg(kHwId);
    const uint32_t xcc = __builtin_amdgcn_s_getreg(kXccId);
    lds[threadIdx.x] = hw;                 // touch the allocation
    for (int i = 0; i < spins; ++i) __builtin_amdgcn_s_sleep(8);
    if ((threadIdx.x & 63) == 0) {         // vector stores only
        const int w = threadIdx.x >> 6;
        const size_t at = ((size_t)blockIdx.x * (blockDim.x >> 6) + w) * 2;
        out[at] = hw;
        out[at + 1] = xcc;
    }
}

int main(int argc, char **argv)
{
    const int nb = argc > 1 ? atoi(argv[1]) : 1152;
    const int nw = argc > 2 ? atoi(argv[2]) : 4;
    const int lb = argc > 3 ? atoi(argv[3]) : 31792;
    if (nb < 1 || nw < 1 || nw > 16 || lb < nw * 64 * 4 || lb > 160 * 1024) {
        fprintf(stderr, "bad arguments\n");
        return 2;
    }
    uint32_t *d;
    const size_t n = (size_t)nb * nw * 2;
    CK(hipMalloc(&d, n * sizeof(uint32_t)));
    CK(hipMemset(d, 0xFF, n * sizeof(uint32_t)));
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(probe),
                           hipFuncAttributeMaxDynamicSharedMemorySize, lb));
    hipLaunchKernelGGL(probe, dim3(nb), dim3(nw * 64), lb, 0, d, 2000);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> h(n);
    CK(hipMemcpy(h.data(), d, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    // per (xcc, se, sh, cu): wave-0 count per SIMD, all waves per SIMD
    std::vector<int> w0(8 * 4 * 2 * 16 * 4, 0), all(8 * 4 * 2 * 16 * 4, 0);
    int hist_simd_w[16][4] = {};
    for (int b = 0; b < nb; ++b)
        for (int w = 0; w < nw; ++w) {
            const uint32_t hw = h[((size_t)b * nw + w) * 2], xcc = h[((size_t)b * nw + w) * 2 + 1] & 7;
            const int simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 3;
            const int key = ((((int)xcc * 4 + se) * 2 + sh) * 16 + cu) * 4 + simd;
            all[key]++;
            if (w == 0) w0[key]++;
            hist_simd_w[w][simd]++;
        }
    printf("wave index -> SIMD histogram (rows: wave within the workgroup)\n");
    for (int w = 0; w < nw; ++w)
        printf("  wave %d: simd0 %5d simd1 %5d simd2 %5d simd3 %5d\n", w, hist_simd_w[w][0],
               hist_simd_w[w][1], hist_simd_w[w][2], hist_simd_w[w][3]);
    int cus = 0, maxw0 = 0, hist_max[17] = {};
    for (size_t c = 0; c < w0.size() / 4; ++c) {
        int tot = 0, mx = 0;
        for (int s = 0; s < 4; ++s) {
            tot += all[c * 4 + s];
            mx = w0[c * 4 + s] > mx ? w0[c * 4 + s] : mx;
        }
        if (!tot) continue;
        ++cus;
        maxw0 = mx > maxw0 ? mx : maxw0;
        hist_max[mx > 16 ? 16 : mx]++;
    }
    printf("CUs used %d; most wave-0s on one SIMD of a CU: %d\n", cus, maxw0);
    printf("CUs by their busiest SIMD's wave-0 count:");
    for (int k = 0; k <= 16; ++k)
        if (hist_max[k]) printf(" %d:%d", k, hist_max[k]);
    printf("\n");
    CK(hipFree(d));
    return 0;
}
