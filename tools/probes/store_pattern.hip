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

// runs: the expansion's real pattern -- a group is a sequence of runs of
// `run` 4-B entries starting at arbitrary 4-B offsets; each run is stored
// as the seg kernels do: up to 3 single entries to the 16-B boundary, 16-B
// stores, up to 3 single entries at the end (RUNFLAT: the same group stored
// as one range, head and tail once per group; LA: the head runs to the next
// 128-B line instead, up to 31 entries)
template <bool RUNFLAT, bool NT = false, bool XCD = false, bool LA = false, int FULL = 0>
__global__ __launch_bounds__(256) void runs_kernel(uint32_t *o, size_t ngroups, int per_group,
                                                   int run)
{
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    size_t nwaves = (size_t)gridDim.x * 4;
    size_t g0 = blockIdx.x * 4 + wv, gend = ngroups;
    if (XCD) {
        // XCD x = block % 8 owns one contiguous eighth of the groups: the
        // line two neighbouring groups share stays in one XCD's L2
        const size_t x = blockIdx.x % 8, gx = (ngroups + 7) / 8;
        nwaves = (size_t)(gridDim.x / 8) * 4;
        g0 = x * gx + (blockIdx.x / 8) * 4 + wv;
        gend = (x + 1) * gx < ngroups ? (x + 1) * gx : ngroups;
    }
    for (size_t g = g0; g < gend; g += nwaves) {
        // groups start 4 B past a boundary and leave the line they share
        // with the next group partly unwritten (FULL 1: whole lines, 144
        // each; FULL 2: groups 4 B past a boundary that cover the buffer, so
        // every line is written whole, the boundary line by two waves)
        const size_t gbase = g * (size_t)per_group + (FULL == 1 ? 0 : 1);
        const int len = per_group - (FULL ? 0 : 2);
        for (int r0 = 0; r0 < len; r0 += RUNFLAT ? len : run) {
            const int total = RUNFLAT ? len : min(run, len - r0);
            uint32_t *p = o + gbase + r0;
            // LA: single entries up to the next 128-B line, so that every
            // wave of 16-B stores covers 8 whole lines (else to 16 B)
            const uint32_t m = LA ? 127u : 15u;
            const int hd = min(total, (int)((((m + 1u) - ((uint32_t)(uintptr_t)p & m)) & m) >> 2));
            if (lane < hd) p[lane] = (uint32_t)lane;
            const int bend = hd + ((total - hd) & ~3);
            for (int t0 = hd; t0 < bend; t0 += 256) {
                const int t = t0 + 4 * lane;
                if (t < bend) {
                    if (NT) {
                        __builtin_nontemporal_store((uint32_t)t, p + t);
                        __builtin_nontemporal_store(1u, p + t + 1);
                        __builtin_nontemporal_store(2u, p + t + 2);
                        __builtin_nontemporal_store(3u, p + t + 3);
                    } else {
                        *reinterpret_cast<uint4 *>(p + t) = make_uint4((uint32_t)t, 1u, 2u, 3u);
                    }
                }
            }
            if (bend + lane < total) p[bend + lane] = 7u;
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
        // the real pattern: 18,432-B groups (64 pairs x 72 entries), runs of 1,728 entries
        const int pg = 4608, nr = (int)(bytes / 4 / pg);
        for (int which = 0; which < 9; ++which) {
            CK(hipEventRecord(a));
            if (which == 0)
                hipLaunchKernelGGL(runs_kernel<false>, dim3(cus * 8), dim3(256), 0, 0,
                                   reinterpret_cast<uint32_t *>(o), (size_t)nr - 1, pg, 1728);
            else if (which == 1)
                hipLaunchKernelGGL(runs_kernel<true>, dim3(cus * 8), dim3(256), 0, 0,
                                   reinterpret_cast<uint32_t *>(o), (size_t)nr - 1, pg, 1728);
            else if (which == 2)
                hipLaunchKernelGGL((runs_kernel<false, true>), dim3(cus * 8), dim3(256), 0, 0,
                                   reinterpret_cast<uint32_t *>(o), (size_t)nr - 1, pg, 1728);
            else if (which == 3)
                hipLaunchKernelGGL((runs_kernel<false, false, true>), dim3(cus * 8), dim3(256), 0, 0,
                                   reinterpret_cast<uint32_t *>(o), (size_t)nr - 1, pg, 1728);
            else if (which == 4)
                hipLaunchKernelGGL((runs_kernel<false, false, false, true>), dim3(cus * 8), dim3(256), 0, 0,
                                   reinterpret_cast<uint32_t *>(o), (size_t)nr - 1, pg, 1728);
            else if (which == 5)
                hipLaunchKernelGGL((runs_kernel<false, false, false, true, 1>), dim3(cus * 8), dim3(256), 0, 0,
                                   reinterpret_cast<uint32_t *>(o), (size_t)nr - 1, pg, 1728);
            else if (which == 6)
                hipLaunchKernelGGL((runs_kernel<true, false, false, true, 1>), dim3(cus * 8), dim3(256), 0, 0,
                                   reinterpret_cast<uint32_t *>(o), (size_t)nr - 1, pg, 1728);
            else if (which == 7)
                hipLaunchKernelGGL((runs_kernel<false, false, false, true, 2>), dim3(cus * 8), dim3(256), 0, 0,
                                   reinterpret_cast<uint32_t *>(o), (size_t)nr - 1, pg, 1728);
            else
                hipLaunchKernelGGL((runs_kernel<false, false, true, true, 2>), dim3(cus * 8), dim3(256), 0, 0,
                                   reinterpret_cast<uint32_t *>(o), (size_t)nr - 1, pg, 1728);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            const double wb = (double)(nr - 1) * (pg - (which >= 5 ? 0 : 2)) * 4.0;
            printf("%-10s %.3f ms  %.2f TB/s\n", which == 0 ? "runs" : which == 1 ? "runs-flat" : which == 2 ? "runs-nt" :
                   which == 3 ? "runs-xcd" : which == 4 ? "runs-line" : which == 5 ? "line-full" :
                   which == 6 ? "flat-full" : which == 7 ? "shared" : "shared-xcd", ms,
                   wb / (ms * 1e-3) / 1e12);
        }
        for (int which = 0; which < 4; ++which) {
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
