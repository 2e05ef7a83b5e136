// Contention probe (round 4): the dependent LDS and L2 round
// trips of the k=48 DFS search wave, measured alone and beside decrement-like
// worker waves in the same workgroup.  Wave 0 runs a dependent chain (an LDS
// read chain, or a chase of 128-B u16 rows in L2 -- the adj16 layout); waves
// 1..S loop the async kernel's worker step until wave 0 is done: 16 row loads
// (u16, 64 lanes, pre-swizzled count indices) then 16 ds_sub_u32 into a
// 4,096-word count block.  Cycles per chain step from s_memtime.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/r4/contention_probe tools/r4/contention_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

constexpr int kWords = 4096;

template <bool L2CHAIN>
__global__ void probe(const uint16_t *rows, const uint16_t *radj, int nrows, int steps, int workers,
                      unsigned long long *out)
{
    __shared__ uint32_t a[kWords];               // the chain's words
    __shared__ uint32_t cnt[kWords];             // the workers' count block
    __shared__ int done;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < kWords; i += blockDim.x) {
        a[i] = (i * 2654435761u) % kWords;
        cnt[i] = 1u << 30;
    }
    if (threadIdx.x == 0) done = 0;
    __syncthreads();
    if (w == 0) {
        int x = (blockIdx.x * 977 + lane) % (L2CHAIN ? nrows : kWords);
        if (L2CHAIN) x = __builtin_amdgcn_readfirstlane(x);
        const unsigned long long t0 = __builtin_readcyclecounter();
        for (int i = 0; i < steps; ++i) {
            if (L2CHAIN) {
                const int v = rows[(size_t)x * 64 + lane];
                x = __builtin_amdgcn_readfirstlane(v);
            } else {
                x = (int)a[(x + lane) & (kWords - 1)];
            }
        }
        const unsigned long long t1 = __builtin_readcyclecounter();
        __hip_atomic_store(&done, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (lane == 0) {
            atomicAdd(&out[0], t1 - t0);
            if (x < 0) out[1] = 2;
        }
    } else if (w <= workers) {
        unsigned it = 0, seed = blockIdx.x * 131 + w * 17;
        while (!__hip_atomic_load(&done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) &&
               it < (1u << 22)) {
            int r[16];
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                seed = seed * 1664525u + 1013904223u;
                r[g] = radj[(size_t)((seed >> 8) % (unsigned)nrows) * 64 + lane];
            }
#pragma unroll
            for (int g = 0; g < 16; ++g) atomicSub(&cnt[r[g] & (kWords - 1)], 1u);
            ++it;
        }
        if (lane == 0) atomicAdd(&out[2], (unsigned long long)it);
    }
}

int main()
{
    const int nrows = 2881, steps = 4000;
    std::vector<uint16_t> h((size_t)nrows * 64), hr((size_t)nrows * 64);
    srand(1);
    for (size_t i = 0; i < h.size(); ++i) {
        h[i] = (uint16_t)(rand() % nrows);
        hr[i] = (uint16_t)(rand() % kWords);
    }
    uint16_t *d, *dr;
    unsigned long long *dout;
    hipMalloc(&d, h.size() * 2);
    hipMalloc(&dr, hr.size() * 2);
    hipMalloc(&dout, 32);
    hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dr, hr.data(), hr.size() * 2, hipMemcpyHostToDevice);
    const int grids[] = {1, 144, 1152};
    const int wk[] = {0, 3, 5};
    for (int chain = 0; chain < 2; ++chain)
        for (int g : grids)
            for (int s : wk) {
                unsigned long long o[4] = {0, 0, 0, 0};
                for (int rep = 0; rep < 2; ++rep) {
                    hipMemset(dout, 0, 32);
                    if (chain)
                        hipLaunchKernelGGL(probe<true>, dim3(g), dim3(64 * (1 + s)), 0, 0, d, dr, nrows,
                                           steps, s, dout);
                    else
                        hipLaunchKernelGGL(probe<false>, dim3(g), dim3(64 * (1 + s)), 0, 0, d, dr, nrows,
                                           steps, s, dout);
                    if (hipDeviceSynchronize() != hipSuccess) {
                        printf("launch failed\n");
                        return 1;
                    }
                }
                hipMemcpy(o, dout, 32, hipMemcpyDeviceToHost);
                printf("%s chain, %4d workgroups, %d worker waves: %.0f cycles per step "
                       "(worker steps per wave %.0f)\n",
                       chain ? "L2 u16-row" : "LDS read", g, s, (double)o[0] / g / steps,
                       s ? (double)o[2] / g / s : 0.0);
            }
    return 0;
}
