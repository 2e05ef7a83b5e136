// calib_traffic.hip -- known-byte calibration of rocprofv3's FETCH_SIZE and
// WRITE_SIZE on gfx950 for the access shapes of the route kernels.
//
// MI355X_MICROARCH.md: FETCH_SIZE = TCC_EA0_RDREQ x 64 B and reports exactly
// half the bytes of a 16-B-per-lane streaming read (128-B requests tallied at
// 64 B); WRITE_SIZE is exact for 16-B-per-lane streaming stores; every other
// width is uncalibrated.  The DFS kernels read u16 rows (one 128-B line per
// wavefront load), gather 4-B port words, and store 4-B table words --
// coalesced (async / runs kernels) or scattered (split-kernel writer).  Each
// kernel below moves a known number of bytes in one of those shapes over a
// 1 GiB buffer (4x the Infinity Cache: every line comes from HBM) after a
// 1 GiB eviction sweep; rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes
// give the counter per dispatch; tools/calib_traffic.py turns the ratios into
// the per-kernel factors of tools/summarize_profile.py.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/calib_traffic tools/calib_traffic.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

static constexpr size_t kBytes = size_t(1) << 30;

__device__ __forceinline__ uint32_t mix(uint64_t i)
{
    uint64_t x = i * 0x9E3779B97F4A7C15ull;
    x ^= x >> 29;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 32;
    return (uint32_t)x;
}

// 16 B per lane, coalesced (the guide's reference shape)
__global__ void calib_read16(const uint4 *p, size_t n, uint32_t *sink)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// one 128-B row (64 lanes x u16) per wavefront load, rows in hashed order:
// the u16 adjacency rows of the async / count / runs DFS kernels
__global__ void calib_rows_u16(const uint16_t *p, size_t nrows, uint32_t *sink, uint32_t key)
{
    const int lane = threadIdx.x & 63;
    const size_t w0 = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
    uint32_t acc = 0;
    for (size_t w = w0; w < nrows; w += nw) {
        const size_t r = mix(w) % nrows;         // a permutation is not needed: bytes are counted per load
        acc = acc * 31u + p[r * 64 + lane];      // not foldable: every load is used
    }
    if (acc == key) sink[0] = acc;
}

// 4 B per lane, coalesced (degree / table reads)
__global__ void calib_read_u32(const uint32_t *p, size_t n, uint32_t *sink)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        acc ^= p[i];
    if (acc == 0x12345678u) sink[0] = acc;
}

// 4-B random gathers (the epilogues' port lookups)
__global__ void calib_gather_u32(const uint32_t *p, size_t n, size_t count, uint32_t *sink)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < count;
         i += (size_t)gridDim.x * blockDim.x)
        acc ^= p[mix(i) % n];
    if (acc == 0x12345678u) sink[0] = acc;
}

// 4 B per lane, coalesced stores (async / runs table epilogues)
__global__ void calib_write_u32(uint32_t *p, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        p[i] = (uint32_t)i;
}

// 4-B scattered stores (the split kernel's writer: a push's children land
// anywhere in the source's row)
__global__ void calib_scatter_u32(uint32_t *p, size_t n, size_t count)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < count;
         i += (size_t)gridDim.x * blockDim.x)
        p[mix(i) % n] = (uint32_t)i;
}

// 16 B per lane stores (the guide's exact shape)
__global__ void calib_write16(uint4 *p, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

__global__ void calib_evict(uint4 *p, size_t n)     // streams a different buffer
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        p[i].x += 1u;
}

int main()
{
    void *a = nullptr, *b = nullptr;
    uint32_t *sink = nullptr;
    CK(hipMalloc(&a, kBytes));
    CK(hipMalloc(&b, kBytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 1, kBytes));
    CK(hipMemset(b, 2, kBytes));
    const dim3 grid(256 * 8), blk(256);
    const size_t n16 = kBytes / 16, n4 = kBytes / 4, nrows = kBytes / 128;
    const size_t gathers = size_t(1) << 22, scatters = size_t(1) << 22;
    auto evict = [&] { hipLaunchKernelGGL(calib_evict, grid, blk, 0, 0, (uint4 *)b, n16); };
    // name, useful bytes, line bytes (128-B lines touched)
    evict();
    hipLaunchKernelGGL(calib_read16, grid, blk, 0, 0, (const uint4 *)a, n16, sink);
    printf("calib_read16 useful=%zu lines=%zu\n", kBytes, kBytes);
    evict();
    hipLaunchKernelGGL(calib_rows_u16, grid, blk, 0, 0, (const uint16_t *)a, nrows, sink, 0x9E3779B9u);
    printf("calib_rows_u16 useful=%zu lines=%zu\n", nrows * 128, nrows * 128);
    evict();
    hipLaunchKernelGGL(calib_read_u32, grid, blk, 0, 0, (const uint32_t *)a, n4, sink);
    printf("calib_read_u32 useful=%zu lines=%zu\n", kBytes, kBytes);
    evict();
    hipLaunchKernelGGL(calib_gather_u32, grid, blk, 0, 0, (const uint32_t *)a, n4, gathers, sink);
    printf("calib_gather_u32 useful=%zu lines=%zu\n", gathers * 4, gathers * 128);
    evict();
    hipLaunchKernelGGL(calib_write_u32, grid, blk, 0, 0, (uint32_t *)a, n4);
    printf("calib_write_u32 useful=%zu lines=%zu\n", kBytes, kBytes);
    evict();
    hipLaunchKernelGGL(calib_scatter_u32, grid, blk, 0, 0, (uint32_t *)a, n4, scatters);
    printf("calib_scatter_u32 useful=%zu lines=%zu\n", scatters * 4, scatters * 128);
    evict();
    hipLaunchKernelGGL(calib_write16, grid, blk, 0, 0, (uint4 *)a, n16);
    printf("calib_write16 useful=%zu lines=%zu\n", kBytes, kBytes);
    CK(hipDeviceSynchronize());
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(sink));
    return 0;
}
