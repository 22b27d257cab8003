/* lz4.c — TEST INFRASTRUCTURE ONLY: CPU restatement of the LZ4 *block* format
 * decoder that Block::from_reader / from_file run for CompressionType::Lz4
 * (src/table/block/mod.rs:104-118, :163-178: lz4_flex::decompress_into into a
 * buffer of header.uncompressed_length bytes).  lz4_flex 0.13 is a third-party
 * crate absent from /root/reference; the block format it decodes is LZ4's
 * published one:
 *   sequence = token (hi nibble literal length, lo nibble match length - 4),
 *              [literal length extension bytes: add each, stop at a byte != 255],
 *              literals, then -- unless the input ends here -- offset u16 LE
 *              (1..written), [match length extension bytes], match copy
 *              (byte by byte, so offset < length repeats the last `offset` bytes).
 * Any overrun of input or output, offset 0 or offset > bytes written, or input
 * ending inside a sequence is an error (Error::Decompress).  Pinned in tests
 * against liblz4 through pyarrow's "lz4_raw" codec (independent implementation).
 * Never linked into the product library. */
#include <stdint.h>
#include <string.h>

#include "lsm_oracle.h"

/* Returns the number of bytes written to dst, or -1 on malformed input. */
int64_t orc_lz4_decompress(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap) {
  uint64_t ip = 0, op = 0;
  if (n == 0) return -1;
  for (;;) {
    if (ip >= n) return -1;
    const uint8_t token = src[ip++];
    uint64_t lit = token >> 4;
    if (lit == 15) {
      uint8_t b;
      do {
        if (ip >= n) return -1;
        b = src[ip++];
        lit += b;
      } while (b == 255);
    }
    if (lit > n - ip || lit > cap - op) return -1;
    memcpy(dst + op, src + ip, lit);
    ip += lit;
    op += lit;
    if (ip == n) return (int64_t)op; /* last sequence: literals only */
    if (n - ip < 2) return -1;
    const uint64_t off = (uint64_t)src[ip] | ((uint64_t)src[ip + 1] << 8);
    ip += 2;
    if (off == 0 || off > op) return -1;
    uint64_t ml = (token & 15u) + 4;
    if ((token & 15u) == 15) {
      uint8_t b;
      do {
        if (ip >= n) return -1;
        b = src[ip++];
        ml += b;
      } while (b == 255);
    }
    if (ml > cap - op) return -1;
    for (uint64_t j = 0; j < ml; ++j) dst[op + j] = dst[op + j - off];
    op += ml;
  }
}
