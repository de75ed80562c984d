/* zgen.c — TEST INFRASTRUCTURE: the host build of the benchmark's seeded input
 * generators (zlib.wasm_amd/csrc/zgpu_gen.h, the same code the device runs in
 * k_generate), so tests can rebuild the exact bytes bench.py compresses and
 * pin them against golden fixtures of the compiled reference. */
#include <stdint.h>
#include <string.h>

#include "../zlib.wasm_amd/csrc/zgpu_gen.h"

/* count buffers of len bytes (len % 4 == 0, dst 4-byte aligned), buffer b is
 * global index first_index + b: the bytes zgpu_generate_dev writes */
int zo_generate(uint8_t *dst, uint64_t len, uint32_t count, int kind, uint64_t seed, uint64_t first_index) {
    if ((len & 3) || ((uintptr_t)dst & 3) || kind < 0 || kind > 5) return -1;
    const uint64_t chunks = (len + ZG_CHUNK - 1) / ZG_CHUNK;
    for (uint32_t b = 0; b < count; b++)
        for (uint64_t c = 0; c < chunks; c++)
            zg_chunk(dst + (uint64_t)b * len + c * ZG_CHUNK, len, kind, seed, first_index + b, c);
    return 0;
}
