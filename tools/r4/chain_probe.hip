// Dependent-chain latency of the DFS search step's instruction mix (round 4):
// ballot -> scalar find-highest -> readlane -> VALU, repeated; plus plain
// VALU and SALU chains.  One wave per CU (the N=8 share's load), s_setprio 3.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/r4/chain_probe tools/r4/chain_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void chain_select(int steps, unsigned long long *out, int *sink)
{
    __builtin_amdgcn_s_setprio(3);
    const int lane = threadIdx.x;
    int x = lane * 7 + blockIdx.x;
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < steps; ++i) {
        const unsigned long long m = __ballot((x & 3) != 0);
        const int h = 63 - __clzll(m | 1ull);
        const int y = __builtin_amdgcn_readlane(x, h);
        x = (x ^ y) + lane;
    }
    unsigned long long t1 = __builtin_readcyclecounter();
    if (lane == 0) atomicAdd(out, t1 - t0);
    if (x == 12345) sink[0] = x;
}

__global__ void chain_valu(int steps, unsigned long long *out, int *sink)
{
    const int lane = threadIdx.x;
    int x = lane;
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < steps; ++i) x = (x * 5 + 3) ^ (x >> 2);
    unsigned long long t1 = __builtin_readcyclecounter();
    if (lane == 0) atomicAdd(out, t1 - t0);
    if (x == 12345) sink[0] = x;
}

__global__ void chain_lds_select(int steps, unsigned long long *out, int *sink)
{
    // an LDS gather feeding a ballot / readlane, the candidate-selection round trip
    __shared__ unsigned words[4096];
    const int lane = threadIdx.x;
    for (int i = lane; i < 4096; i += 64) words[i] = i * 2654435761u;
    __syncthreads();
    int x = lane;
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < steps; ++i) {
        const unsigned w = words[(x * 33 + lane) & 4095];
        const unsigned long long m = __ballot(w & 1u);
        const int h = 63 - __clzll(m | 1ull);
        x = __builtin_amdgcn_readlane((int)w, h) & 4095;
    }
    unsigned long long t1 = __builtin_readcyclecounter();
    if (lane == 0) atomicAdd(out, t1 - t0);
    if (x == 12345) sink[0] = x;
}

int main()
{
    unsigned long long *d;
    int *sink;
    hipMalloc(&d, 8);
    hipMalloc(&sink, 4);
    const int steps = 4000;
    const int grids[] = {1, 256};
    const char *names[] = {"ballot->s_flbit->readlane->valu", "dependent valu (mul/xor/shift)",
                           "lds gather->ballot->readlane"};
    for (int k = 0; k < 3; ++k)
        for (int g : grids) {
            unsigned long long h = 0;
            for (int rep = 0; rep < 2; ++rep) {
                hipMemset(d, 0, 8);
                if (k == 0) hipLaunchKernelGGL(chain_select, dim3(g), dim3(64), 0, 0, steps, d, sink);
                else if (k == 1) hipLaunchKernelGGL(chain_valu, dim3(g), dim3(64), 0, 0, steps, d, sink);
                else hipLaunchKernelGGL(chain_lds_select, dim3(g), dim3(64), 0, 0, steps, d, sink);
                hipDeviceSynchronize();
            }
            hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
            printf("%-36s %3d waves: %.1f cycles per step\n", names[k], g, (double)h / g / steps);
        }
    return 0;
}
