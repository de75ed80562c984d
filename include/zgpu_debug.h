/*
 * zgpu_debug.h — test-only stage access (not part of the drop-in ABI).
 *
 * Runs the first deflate stages on ONE host buffer and copies the
 * position-indexed intermediates back, so tests can compare each GPU stage
 * with the oracle's position-parallel formulation (oracle/zoracle.h
 * zo_pp_links / zo_pp_match).  link: n x u16; rfull, rquart: n x u32 (levels
 * 4..9; rquart only for levels 5..9, may be NULL).  Returns ZGPU_OK or an
 * error code.
 */
#ifndef ZGPU_DEBUG_H
#define ZGPU_DEBUG_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
int zgpu_debug_stages(const uint8_t *src, size_t n, int level, uint16_t *link,
                      uint32_t *rfull, uint32_t *rquart);
/* streams the block-parallel decode of a lone stream finished so far (the
 * others went through the sequential decode) */
uint64_t zgpu_debug_par_inflates(void);
/* buffers the segmented lazy parse (k_parse_seg) handed to the sequential one
 * so far: out[0] lanes that did not meet their neighbour within one segment,
 * out[1] run-ons longer than the lane's staging room */
int zgpu_debug_parse_fallbacks(uint64_t *out);
#ifdef __cplusplus
}
#endif
#endif
