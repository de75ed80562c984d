// zgpu_gen.hip — seeded synthetic workloads, generated in HBM.
// Inputs of the benchmark configs are far too large to stage over PCIe inside a
// timed loop, so they are produced on the device.  The generators themselves
// live in zgpu_gen.h, shared with the host build the tests use to rebuild (and
// golden-pin) the same bytes; one thread writes one 4 KiB chunk.
#include "zgpu_internal.h"
#include "zgpu_gen.h"

namespace zgpu {

__global__ void k_generate(uint8_t *dst, uint64_t len, uint32_t count, int kind, uint64_t seed,
                           uint64_t first_index) {
    const uint64_t chunks_per = (len + ZG_CHUNK - 1) / ZG_CHUNK;
    const uint64_t total = chunks_per * count;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < total;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t b = t / chunks_per, c = t % chunks_per;
        zg_chunk(dst + b * len + c * ZG_CHUNK, len, kind, seed, first_index + b, c);
    }
}

int launch_generate(uint8_t *dst, uint64_t len, uint32_t count, int kind, uint64_t seed,
                    uint64_t first_index, hipStream_t st) {
    if (count == 0 || len == 0) return 0;
    if ((len & 3) || (reinterpret_cast<uintptr_t>(dst) & 3) || kind < 0 || kind > 5)
        return (int)hipErrorInvalidValue;
    const uint64_t total = ((len + ZG_CHUNK - 1) / ZG_CHUNK) * count;
    uint64_t blocks = (total + 255) / 256;
    if (blocks > 65535) blocks = 65535;
    hipLaunchKernelGGL(k_generate, dim3((uint32_t)blocks), dim3(256), 0, st, dst, len, count, kind,
                       seed, first_index);
    return (int)hipGetLastError();
}

}  // namespace zgpu
