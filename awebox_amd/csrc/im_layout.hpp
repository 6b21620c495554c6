// Instance-minor layout helpers shared by the evaluators' generated paths (awempc.hip, awedual.hip).
//
// An instance-minor buffer holds row i of every instance side by side: X[i * ld + b].  A wavefront
// with lane = instance then reads or writes one 512-byte row per access.  Rows are addressed as a
// uniform byte offset row * ld8 (32-bit; the hosts keep every such buffer below 4 GiB) plus the
// lane's constant offset lb = 8 b, so an access is one scalar base plus a vector offset.
#pragma once

#include <hip/hip_runtime.h>

namespace im {

__device__ __forceinline__ const double& at(const double* x, unsigned row, unsigned ld8, unsigned lb) {
    return *reinterpret_cast<const double*>(reinterpret_cast<const char*>(x) + row * ld8 + lb);
}
__device__ __forceinline__ double& at(double* x, unsigned row, unsigned ld8, unsigned lb) {
    return *reinterpret_cast<double*>(reinterpret_cast<char*>(x) + row * ld8 + lb);
}
__device__ __forceinline__ double& at_byte(double* x, unsigned off) {
    return *reinterpret_cast<double*>(reinterpret_cast<char*>(x) + off);
}

// blockIdx.x -> tile: consecutive tiles to the same XCD (blocks are dealt to the 8 XCDs round robin),
// so that the tiles of one instance block share that XCD's L2
__device__ __forceinline__ int xcd_tile(int total) {
    const int per = (total + 7) / 8;
    return (blockIdx.x & 7) * per + (blockIdx.x >> 3);
}
__host__ __device__ constexpr int xcd_grid(int total) { return ((total + 7) / 8) * 8; }

// A [batch][na] and B [batch][nb] (per-instance rows) -> AT[i * ld + b], BT[i * ld + b], 64 x 64 tiles
// through LDS; grid (ceil((na + nb) / 64), ceil(batch / 64)), 256 threads
__global__ __launch_bounds__(256) void transpose_in_kernel(const double* __restrict__ A, const double* __restrict__ B,
                                                           double* __restrict__ AT, double* __restrict__ BT,
                                                           int batch, int na, int nb, int ld) {
    __shared__ double tile[64][65];
    const int ncol = na + nb;
    const int c0 = blockIdx.x * 64, b0 = blockIdx.y * 64;
    const int tid = threadIdx.x;
    double r[16];
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        const int e = tid + it * 256, bl = e >> 6, cl = e & 63;
        const int bc = min(b0 + bl, batch - 1), cc = min(c0 + cl, ncol - 1);   // unconditional loads
        r[it] = cc < na ? A[(size_t)bc * na + cc] : B[(size_t)bc * nb + (cc - na)];
    }
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        const int e = tid + it * 256;
        tile[e >> 6][e & 63] = r[it];
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        const int e = tid + it * 256, cl = e >> 6, bl = e & 63;
        const int b = b0 + bl, c = c0 + cl;
        if (b < batch && c < ncol) {
            if (c < na) AT[(size_t)c * ld + b] = tile[bl][cl];
            else BT[(size_t)(c - na) * ld + b] = tile[bl][cl];
        }
    }
}

// stages n destination-table entries into LDS as byte offsets (pos * row8), 8 loads in flight per thread
template <int NT>
__device__ __forceinline__ void stage_offsets(unsigned* dst, const unsigned* src, int n, unsigned row8, int tid) {
    for (int base = tid; base < n; base += NT * 8) {
        unsigned r[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) r[u] = src[base + u * NT < n ? base + u * NT : n - 1];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (base + u * NT < n) dst[base + u * NT] = r[u] * row8;
    }
}

}  // namespace im
