// HBM read-bandwidth probe: XOR-reduce a 4 GiB buffer with 16-byte loads
// (the ceiling the checksum kernels are measured against).  Not product code.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(256) void rd(const uint4 *__restrict__ p, size_t n16, uint32_t *out, int unroll) {
    uint32_t acc = 0;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        uint4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
        acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
    }
    for (; i < n16; i += stride) { uint4 a = p[i]; acc ^= a.x ^ a.y ^ a.z ^ a.w; }
    if (acc == 0x12345678u) out[0] = acc;
}
// the access shape of k_crc32s<16>: 16 lanes per 4 KiB buffer, lane l reads
// the 64 bytes at 64 l of every 1 KiB row as four 16-byte loads (kContig:
// the four loads of a row at 16 l + 256 q instead, 256 contiguous bytes per
// 16-lane group and instruction)
template <bool kContig>
__global__ __launch_bounds__(1024) void rd_rows(const uint8_t *__restrict__ p, size_t nbuf, uint32_t *out) {
    const int lane = threadIdx.x & 15;
    const size_t groups = (size_t)gridDim.x * (blockDim.x / 16);
    uint32_t acc = 0;
    for (size_t b = (size_t)blockIdx.x * (blockDim.x / 16) + threadIdx.x / 16; b < nbuf; b += groups) {
        const uint8_t *buf = p + (b << 12);
        for (int r = 0; r < 4; r += 2) {
            uint4 v[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int row = r + (k >> 2), q = k & 3;
                const size_t o = (size_t)row * 1024 + (kContig ? 16 * lane + 256 * q : 64 * lane + 16 * q);
                v[k] = *reinterpret_cast<const uint4 *>(buf + o);
            }
#pragma unroll
            for (int k = 0; k < 8; k++) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}
int main() {
    const size_t bytes = 4ull << 30;
    uint4 *p; uint32_t *o;
    hipMalloc(&p, bytes); hipMalloc(&o, 4); hipMemset(p, 1, bytes);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int grid : {1024, 2048, 4096, 8192, 16384}) {
        hipLaunchKernelGGL(rd, dim3(grid), dim3(256), 0, 0, p, bytes / 16, o, 4);
        hipEventRecord(e0);
        for (int r = 0; r < 5; r++) hipLaunchKernelGGL(rd, dim3(grid), dim3(256), 0, 0, p, bytes / 16, o, 4);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("grid %d: %.2f TB/s\n", grid, 5.0 * bytes / (ms / 1e3) / 1e12);
    }
    for (int contig = 0; contig < 2; contig++)
        for (int grid : {512, 1024, 2048}) {
            auto k = contig ? rd_rows<true> : rd_rows<false>;
            hipLaunchKernelGGL(k, dim3(grid), dim3(1024), 0, 0, (const uint8_t *)p, bytes >> 12, o);
            hipEventRecord(e0);
            for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k, dim3(grid), dim3(1024), 0, 0, (const uint8_t *)p, bytes >> 12, o);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            printf("rows %s grid %d: %.2f TB/s\n", contig ? "contiguous" : "crc32s-strided", grid, 5.0 * bytes / (ms / 1e3) / 1e12);
        }
    return 0;
}
