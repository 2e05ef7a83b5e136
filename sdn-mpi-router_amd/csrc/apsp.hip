// apsp.hip -- all-pairs hop distances by blocked min-plus closure.
//
// For small dense fabrics (fat-tree k<=48, dragonfly) the all-pairs hop
// matrix fits in HBM many times over (V=2880: 16.6 MB of uint16) and the
// blocked Floyd-Warshall closure D <- min(D, D[:,K] (+) D[K,:]) over 64-wide
// pivot blocks is a tiled min-plus "GEMM".  min-plus is not a multiply-add,
// so it runs on the VALU (v_add/v_min), not MFMA: each thread owns a 4x4
// output micro-tile, pivot row/column tiles are staged in LDS and read as
// broadcasts.  Three phases per pivot block: (1) the pivot tile closes on
// itself, (2) pivot row and column tiles close against it, (3) every other
// tile takes one min-plus product.  Distances saturate at 0xFFFF (= no
// path), the same convention as the msbfs dist tables it cross-checks.
#include "common.h"

namespace {

constexpr int T = 64;            // tile edge
constexpr uint32_t INF = 0xFFFFu;

__device__ __forceinline__ uint32_t sat_add(uint32_t a, uint32_t b)
{
    const uint32_t c = a + b;
    return c > INF ? INF : c;
}

__global__ __launch_bounds__(256) void apsp_init_kernel(
    int V, int Vp, const int32_t *__restrict__ row_ptr,
    const int32_t *__restrict__ col, uint16_t *__restrict__ D)
{
    const size_t n = (size_t)Vp * Vp;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const int r = (int)(i / Vp), c = (int)(i % Vp);
        D[i] = (r == c && r < V) ? 0 : (uint16_t)INF;
    }
}

__global__ __launch_bounds__(256) void apsp_edges_kernel(
    int V, int Vp, const int32_t *__restrict__ row_ptr,
    const int32_t *__restrict__ col, uint16_t *__restrict__ D)
{
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= V) return;
    for (int e = row_ptr[u]; e < row_ptr[u + 1]; ++e)
        if (col[e] != u) D[(size_t)u * Vp + col[e]] = 1;
}

// phase 1: the pivot tile, 64 sequential pivots inside LDS
__global__ __launch_bounds__(256) void apsp_phase1_kernel(int Vp, int kb, uint16_t *__restrict__ D)
{
    __shared__ uint32_t t[T][T + 1];
    const int base = kb * T;
    for (int i = threadIdx.x; i < T * T; i += 256)
        t[i / T][i % T] = D[(size_t)(base + i / T) * Vp + base + i % T];
    __syncthreads();
    for (int k = 0; k < T; ++k) {
        for (int i = threadIdx.x; i < T * T; i += 256) {
            const int r = i / T, c = i % T;
            const uint32_t v = sat_add(t[r][k], t[k][c]);
            if (v < t[r][c]) t[r][c] = v;
        }
        __syncthreads();
    }
    for (int i = threadIdx.x; i < T * T; i += 256)
        D[(size_t)(base + i / T) * Vp + base + i % T] = (uint16_t)t[i / T][i % T];
}

// phase 2: blockIdx.y == 0 -> pivot row tile (kb, j), 1 -> column tile (j, kb)
__global__ __launch_bounds__(256) void apsp_phase2_kernel(int Vp, int kb, uint16_t *__restrict__ D)
{
    int j = blockIdx.x;
    if (j >= kb) ++j;                       // skip the pivot tile itself
    const bool row = blockIdx.y == 0;
    __shared__ uint32_t piv[T][T + 1];
    __shared__ uint32_t t[T][T + 1];
    const int pb = kb * T;
    const int r0 = row ? pb : j * T;
    const int c0 = row ? j * T : pb;
    for (int i = threadIdx.x; i < T * T; i += 256) {
        piv[i / T][i % T] = D[(size_t)(pb + i / T) * Vp + pb + i % T];
        t[i / T][i % T] = D[(size_t)(r0 + i / T) * Vp + c0 + i % T];
    }
    __syncthreads();
    for (int k = 0; k < T; ++k) {
        for (int i = threadIdx.x; i < T * T; i += 256) {
            const int r = i / T, c = i % T;
            const uint32_t v = row ? sat_add(piv[r][k], t[k][c]) : sat_add(t[r][k], piv[k][c]);
            if (v < t[r][c]) t[r][c] = v;
        }
        __syncthreads();
    }
    for (int i = threadIdx.x; i < T * T; i += 256)
        D[(size_t)(r0 + i / T) * Vp + c0 + i % T] = (uint16_t)t[i / T][i % T];
}

// phase 3: tile (bi, bj) = min(tile, A(bi,kb) (+) B(kb,bj)); 4x4 per thread
__global__ __launch_bounds__(256) void apsp_phase3_kernel(int Vp, int kb, uint16_t *__restrict__ D)
{
    int bi = blockIdx.y, bj = blockIdx.x;
    if (bi >= kb) ++bi;
    if (bj >= kb) ++bj;
    __shared__ uint32_t A[T][T + 1];   // A[r][k]
    __shared__ uint32_t B[T][T + 1];   // B[k][c]
    const int pb = kb * T;
    for (int i = threadIdx.x; i < T * T; i += 256) {
        A[i / T][i % T] = D[(size_t)(bi * T + i / T) * Vp + pb + i % T];
        B[i / T][i % T] = D[(size_t)(pb + i / T) * Vp + bj * T + i % T];
    }
    __syncthreads();
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    uint32_t acc[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c)
            acc[r][c] = D[(size_t)(bi * T + ty * 4 + r) * Vp + bj * T + tx * 4 + c];
#pragma unroll 8
    for (int k = 0; k < T; ++k) {
        uint32_t a[4], b[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) a[r] = A[ty * 4 + r][k];
#pragma unroll
        for (int c = 0; c < 4; ++c) b[c] = B[k][tx * 4 + c];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[r][c] = min(acc[r][c], a[r] + b[c]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c)
            D[(size_t)(bi * T + ty * 4 + r) * Vp + bj * T + tx * 4 + c] =
                (uint16_t)(acc[r][c] > INF ? INF : acc[r][c]);
}

}  // namespace

int sdnr_launch_apsp(sdnr_ctx *ctx, uint16_t *d_dist)
{
    const int V = ctx->V;
    if (V == 0) return SDNR_OK;
    if (V > 16384) return sdnr_fail(SDNR_ERR_INVAL, "apsp: V=%d > 16384", V);
    const int nb = (V + T - 1) / T;
    const int Vp = nb * T;
    const size_t bytes = (size_t)Vp * Vp * sizeof(uint16_t);
    uint16_t *D = d_dist;
    if (Vp != V) {
        int rc = sdnr_reserve(&ctx->scratch, &ctx->scratch_bytes, bytes);
        if (rc) return rc;
        D = static_cast<uint16_t *>(ctx->scratch);
    }
    ctx->last_kernel = "apsp_phase{1,2,3}_kernel";
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev0, ctx->stream));
    hipLaunchKernelGGL(apsp_init_kernel, dim3(1024), dim3(256), 0, ctx->stream, V, Vp,
                       ctx->row_ptr, ctx->col, D);
    hipLaunchKernelGGL(apsp_edges_kernel, dim3((V + 255) / 256), dim3(256), 0, ctx->stream,
                       V, Vp, ctx->row_ptr, ctx->col, D);
    for (int kb = 0; kb < nb; ++kb) {
        hipLaunchKernelGGL(apsp_phase1_kernel, dim3(1), dim3(256), 0, ctx->stream, Vp, kb, D);
        if (nb > 1) {
            hipLaunchKernelGGL(apsp_phase2_kernel, dim3(nb - 1, 2), dim3(256), 0, ctx->stream,
                               Vp, kb, D);
            hipLaunchKernelGGL(apsp_phase3_kernel, dim3(nb - 1, nb - 1), dim3(256), 0,
                               ctx->stream, Vp, kb, D);
        }
    }
    SDNR_HIP(hipGetLastError());
    if (D != d_dist)
        SDNR_HIP(hipMemcpy2DAsync(d_dist, (size_t)V * 2, D, (size_t)Vp * 2, (size_t)V * 2, V,
                                  hipMemcpyDeviceToDevice, ctx->stream));
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
    return SDNR_OK;
}
