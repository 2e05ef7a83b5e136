// Dependent-load latency probe (round 4): how long does one row fetch of the
// k=48 DFS chain take?  A wave chases a pseudo-random sequence of 128-B rows
// (u16 x 64, the adj16 layout) or 512-B rows (u64 x 64, a bitmap layout):
// the next row id comes from the loaded data, so every step waits for its
// load.  Cycles per step from s_memtime around the chase.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/r4/latency_probe tools/r4/latency_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <vector>

__global__ void chase16(const uint16_t *rows, int nrows, int steps, int warm, unsigned long long *out)
{
    const int lane = threadIdx.x;
    if (warm) {                                  // touch every line of the array first
        for (int i = lane; i < nrows * 64; i += 64 * 64)
            if (rows[i] == 0xFFFF) out[1] = 1;
    }
    int x = (blockIdx.x * 977) % nrows;
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < steps; ++i) {
        const int v = rows[(size_t)x * 64 + lane];
        x = __builtin_amdgcn_readfirstlane(v);
    }
    unsigned long long t1 = __builtin_readcyclecounter();
    if (lane == 0) { atomicAdd(&out[0], t1 - t0); if (x < 0) out[1] = 2; }
}

__global__ void chase64(const uint64_t *rows, int nrows, int steps, int warm, unsigned long long *out)
{
    const int lane = threadIdx.x;
    if (warm) {
        for (int i = lane; i < nrows * 64; i += 64 * 16)
            if (rows[i] == ~0ull) out[1] = 1;
    }
    int x = (blockIdx.x * 977) % nrows;
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < steps; ++i) {
        const uint64_t v = rows[(size_t)x * 64 + lane];
        x = __builtin_amdgcn_readfirstlane((int)(v & 0xFFFFFFFF));
    }
    unsigned long long t1 = __builtin_readcyclecounter();
    if (lane == 0) { atomicAdd(&out[0], t1 - t0); if (x < 0) out[1] = 2; }
}

__global__ void chase_lds(int steps, unsigned long long *out)
{
    __shared__ uint32_t a[4096];
    const int lane = threadIdx.x;
    for (int i = lane; i < 4096; i += 64) a[i] = (i * 2654435761u) % 4096u;
    __syncthreads();
    int x = lane;
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < steps; ++i) x = (int)a[(x + lane) & 4095];
    unsigned long long t1 = __builtin_readcyclecounter();
    if (lane == 0) { atomicAdd(&out[0], t1 - t0); if (x < 0) out[1] = 2; }
}

int main()
{
    const int nrows = 2881, steps = 2000;
    std::vector<uint16_t> h16((size_t)nrows * 64);
    std::vector<uint64_t> h64((size_t)nrows * 64);
    srand(1);
    for (size_t i = 0; i < h16.size(); ++i) {
        const int r = rand() % nrows;
        h16[i] = (uint16_t)r;
        h64[i] = (uint64_t)r;
    }
    uint16_t *d16; uint64_t *d64; unsigned long long *dout;
    hipMalloc(&d16, h16.size() * 2); hipMalloc(&d64, h64.size() * 8); hipMalloc(&dout, 16);
    hipMemcpy(d16, h16.data(), h16.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(d64, h64.data(), h64.size() * 8, hipMemcpyHostToDevice);
    int grids[] = {1, 144, 1152};
    for (int g : grids)
        for (int warm = 0; warm < 2; ++warm) {
            for (int kind = 0; kind < 2; ++kind) {
                unsigned long long h[2] = {0, 0};
                for (int rep = 0; rep < 3; ++rep) {   // last of 3 launches
                    hipMemset(dout, 0, 16);
                    if (kind == 0) hipLaunchKernelGGL(chase16, dim3(g), dim3(64), 0, 0, d16, nrows, steps, warm, dout);
                    else hipLaunchKernelGGL(chase64, dim3(g), dim3(64), 0, 0, d64, nrows, steps, warm, dout);
                    hipDeviceSynchronize();
                }
                hipMemcpy(h, dout, 16, hipMemcpyDeviceToHost);
                printf("%s rows, %4d waves, warm=%d: %.0f cycles per dependent row load\n",
                       kind == 0 ? "u16 128-B" : "u64 512-B", g, warm, (double)h[0] / g / steps);
            }
        }
    for (int g : grids) {
        unsigned long long h[2] = {0, 0};
        hipMemset(dout, 0, 16);
        hipLaunchKernelGGL(chase_lds, dim3(g), dim3(64), 0, 0, steps, dout);
        hipDeviceSynchronize();
        hipMemcpy(h, dout, 16, hipMemcpyDeviceToHost);
        printf("LDS ds_read_b32 chain, %4d waves: %.0f cycles per step\n", g, (double)h[0] / g / steps);
    }
    return 0;
}
