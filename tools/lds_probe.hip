// LDS access probe (tools only, not shipped): random 4-byte reads from a byte
// array in LDS, as a chain walk would issue them.
//   mode 0: aligned ds_read_b32 at a random word
//   mode 1: ds_read_b32 at a random BYTE address (unaligned access mode)
//   mode 2: the same 4 bytes from two aligned reads + v_alignbyte_b32
//   mode 3: ds_read_u16 at a random byte address
// Reports whether mode 1/3 return the right bytes and the cycles per
// wave-read with 16 waves per CU issuing 8 independent reads per round.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

constexpr int kBytes = 36 * 1024;

__device__ inline uint32_t rnd(uint32_t &s) { s ^= s << 13; s ^= s >> 17; s ^= s << 5; return s; }

template <int kMode>
__global__ __launch_bounds__(1024) void probe(uint32_t *out, uint64_t *cyc, int rounds, uint32_t *bad) {
    __shared__ __attribute__((aligned(16))) uint8_t B[kBytes + 64];
    for (int i = threadIdx.x; i < (kBytes + 64) / 4; i += 1024)
        reinterpret_cast<uint32_t *>(B)[i] = (uint32_t)(i * 2654435761u);
    __syncthreads();
    uint32_t s = 0x9e3779b9u ^ (threadIdx.x * 747796405u) ^ blockIdx.x;
    uint32_t acc = 0;
    const uint64_t t0 = wall_clock64();
    for (int r = 0; r < rounds; r++) {
        uint32_t a[8], v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) a[k] = (rnd(s) ^ acc) % kBytes;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if (kMode == 0) v[k] = reinterpret_cast<const uint32_t *>(B)[a[k] >> 2];
            else if (kMode == 1) {
                uint32_t x;
                asm volatile("ds_read_b32 %0, %1" : "=v"(x) : "v"((uint32_t)(uintptr_t)(B + a[k])));
                v[k] = x;
            } else if (kMode == 2) {
                const uint32_t *w = reinterpret_cast<const uint32_t *>(B + (a[k] & ~3u));
                v[k] = __builtin_amdgcn_alignbyte(w[1], w[0], a[k] & 3u);
            } else {
                uint32_t x;
                asm volatile("ds_read_u16 %0, %1" : "=v"(x) : "v"((uint32_t)(uintptr_t)(B + a[k])));
                v[k] = x;
            }
        }
        if (kMode == 1 || kMode == 3) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if (kMode == 1 || kMode == 3) {
                const uint32_t *w = reinterpret_cast<const uint32_t *>(B + (a[k] & ~3u));
                uint32_t want = __builtin_amdgcn_alignbyte(w[1], w[0], a[k] & 3u);
                if (kMode == 3) want &= 0xffffu;
                if (want != v[k]) atomicAdd(bad, 1u);
            }
            acc += v[k];
        }
    }
    const uint64_t t1 = wall_clock64();
    out[blockIdx.x * 1024 + threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int kMode>
static void run(int nblk, int rounds) {
    uint32_t *out, *bad;
    uint64_t *cyc;
    hipMalloc(&out, nblk * 1024 * 4);
    hipMalloc(&cyc, nblk * 8);
    hipMalloc(&bad, 4);
    hipMemset(bad, 0, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    probe<kMode><<<nblk, 1024>>>(out, cyc, 4, bad);
    hipDeviceSynchronize();
    hipMemset(bad, 0, 4);
    hipEventRecord(e0);
    probe<kMode><<<nblk, 1024>>>(out, cyc, rounds, bad);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    uint32_t b;
    hipMemcpy(&b, bad, 4, hipMemcpyDeviceToHost);
    // wave-reads per CU: 16 waves x rounds x 8; at ~2.4 GHz
    const double per_cu = 16.0 * rounds * 8 * nblk / 256.0;
    printf("mode %d: %.3f ms, %.2f ns per wave-read per CU (%.2f cycles at 2.4 GHz), wrong %u\n", kMode, ms,
           ms * 1e6 / per_cu, ms * 1e6 / per_cu * 2.4, b);
    hipFree(out);
    hipFree(cyc);
    hipFree(bad);
}

int main() {
    const int nblk = 256 * 4, rounds = 4096;
    run<0>(nblk, rounds);
    run<1>(nblk, rounds);
    run<2>(nblk, rounds);
    run<3>(nblk, rounds);
    return 0;
}
