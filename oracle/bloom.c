/* bloom.c — TEST INFRASTRUCTURE ONLY: CPU restatement of the reference's
 * standard Bloom filter (the table's "filter" section), used as the checker
 * for lsm_bloom_* in tests/.  Never linked into the product library.
 *
 *   orc_bloom_shape_bpk   <- Builder::with_bpk      src/table/filter/standard_bloom/builder.rs:91-126
 *   orc_bloom_shape_fpr   <- Builder::with_fp_rate  builder.rs:58-85, calculate_m :128-151
 *   orc_bloom_build       <- set_with_hash + build  builder.rs:33-53,154-170; bit_array/builder.rs:8-11,38-45
 *   orc_bloom_contains    <- contains_hash          standard_bloom/mod.rs:100-120; bit_array/reader.rs:8-13,33-40
 *
 * Arithmetic follows the Rust source literally: f32 throughout the shape
 * computation (`as usize` truncates toward zero and saturates), u64 wrapping
 * arithmetic for the double hashing. */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "lsm_oracle.h"

static const float kLn2 = 0.693147180559945309417232121458176568f; /* std::f32::consts::LN_2 */

static uint64_t f32_to_usize(float x) { /* Rust `as usize`: trunc, NaN/neg -> 0, saturate */
  if (!(x > 0.0f)) return 0;
  if (x >= 18446744073709551616.0f) return UINT64_MAX;
  return (uint64_t)x;
}

/* builder.rs:128-151 */
uint64_t orc_bloom_calculate_m(uint64_t n, float fpr) {
  const float nf = (float)n;
  const float ln2_sq = kLn2 * kLn2; /* LN_2.powi(2) */
  const float numerator = nf * logf(fpr);
  const float m = -(numerator / ln2_sq);
  return f32_to_usize(ceilf(m / 8.0f) * 8.0f);
}

/* builder.rs:58-85 */
int orc_bloom_shape_fpr(uint64_t n, float fpr, uint64_t* m, uint64_t* k) {
  if (n == 0) return -1; /* assert!(n > 0) */
  if (!(fpr >= 0.0000001f)) fpr = 0.0000001f; /* fpr.max(0.000_000_1) */
  const uint64_t mm = orc_bloom_calculate_m(n, fpr);
  const float bpk = (float)(mm / n);
  uint64_t kk = f32_to_usize(bpk * kLn2);
  *m = mm;
  *k = kk < 1 ? 1 : kk;
  return 0;
}

/* builder.rs:91-126 */
int orc_bloom_shape_bpk(uint64_t n, float bpk, uint64_t* m, uint64_t* k) {
  if (!(bpk > 0.0f) || n == 0) return -1;
  const uint64_t mm = n * f32_to_usize(bpk);
  uint64_t kk = f32_to_usize(bpk * kLn2);
  const uint64_t bytes = f32_to_usize(ceilf((float)mm / 8.0f));
  *m = bytes * 8;
  *k = kk < 1 ? 1 : kk;
  return 0;
}

/* builder.rs:10-13 (fastbloom's secondary hash) */
static uint64_t secondary_hash(uint64_t h1) { return (h1 >> 32) * 0x517cc1b727220a95ULL; }

/* Full filter bytes (builder.rs:33-53): MAGIC "LSM\x03", filter type 0
 * (StandardBloom, filter/mod.rs:64-89), hash type 0, m u64 LE, k u64 LE, then
 * m/8 bit-array bytes (bit i = byte i/8, mask 0x80 >> i%8).  out holds
 * ORC_BLOOM_HDR + m/8 bytes. */
void orc_bloom_build(const uint64_t* hashes, uint64_t n, uint64_t m, uint64_t k, uint8_t* out) {
  static const uint8_t magic[4] = {'L', 'S', 'M', 3};
  memcpy(out, magic, 4);
  out[4] = 0;
  out[5] = 0;
  for (int b = 0; b < 8; ++b) out[6 + b] = (uint8_t)(m >> (8 * b));
  for (int b = 0; b < 8; ++b) out[14 + b] = (uint8_t)(k >> (8 * b));
  uint8_t* bits = out + ORC_BLOOM_HDR;
  memset(bits, 0, m / 8);
  if (m == 0) return; /* the reference panics at h1 % 0 (BitsPerKey < 1): no bits to set */
  for (uint64_t j = 0; j < n; ++j) {
    uint64_t h1 = hashes[j], h2 = secondary_hash(h1);
    for (uint64_t i = 1; i <= k; ++i) {
      const uint64_t idx = h1 % m;
      bits[idx / 8] |= (uint8_t)(0x80u >> (idx % 8));
      h1 += h2;
      h2 *= i;
    }
  }
}

/* StandardBloomFilterReader::new + contains_hash (mod.rs:36-86, :100-120).
 * Returns 1 (may contain), 0 (absent), -1 malformed header. */
int orc_bloom_contains(const uint8_t* filter, uint64_t len, uint64_t h1) {
  if (len < ORC_BLOOM_HDR || memcmp(filter, "LSM\x03", 4) != 0 || filter[4] != 0 || filter[5] != 0) return -1;
  uint64_t m = 0, k = 0;
  for (int b = 7; b >= 0; --b) m = (m << 8) | filter[6 + b];
  for (int b = 7; b >= 0; --b) k = (k << 8) | filter[14 + b];
  if (m == 0 || (m + 7) / 8 > len - ORC_BLOOM_HDR) return -1;
  const uint8_t* bits = filter + ORC_BLOOM_HDR;
  uint64_t h2 = secondary_hash(h1);
  for (uint64_t i = 1; i <= k; ++i) {
    const uint64_t idx = h1 % m;
    if (!(bits[idx / 8] & (0x80u >> (idx % 8)))) return 0;
    h1 += h2;
    h2 *= i;
  }
  return 1;
}
