/*
 * xxh3.c — TEST INFRASTRUCTURE ONLY (see lsm_oracle.h).
 *
 * Scalar restatement of XXH3-64 / XXH3-128 (seed 0, default 192-byte secret),
 * the algorithm xxhash-rust ^0.8.15 implements and the reference calls at
 *   src/hash.rs:2-9                     hash64 / hash128
 *   src/table/block/mod.rs:70,94,141    payload checksum
 *   src/table/block/header.rs:13-45     header checksum (streaming digest128)
 *   src/table/block/hash_index/mod.rs:35-41  bucket position (hash64)
 * Pinned by src/hash.rs:17-31 KATs and python-xxhash (tests/test_oracle.py).
 */
#include "lsm_oracle.h"

#include <string.h>
#ifdef __AVX2__
#include <immintrin.h>
#endif

static const uint8_t kSecret[192] = {
    0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c, 0xf7, 0x21, 0xad, 0x1c,
    0xde, 0xd4, 0x6d, 0xe9, 0x83, 0x90, 0x97, 0xdb, 0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3, 0x67, 0x1f,
    0xcb, 0x79, 0xe6, 0x4e, 0xcc, 0xc0, 0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc, 0xff, 0x72, 0x21,
    0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0, 0x35, 0x90, 0xe6, 0x81, 0x3a, 0x26, 0x4c,
    0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb, 0x88, 0xd0, 0x65, 0x8b, 0x1b, 0x53, 0x2e, 0xa3,
    0x71, 0x64, 0x48, 0x97, 0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19, 0xef, 0x46, 0xa9, 0xde, 0xac, 0xd8,
    0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9, 0xdc, 0xbb, 0xc7, 0xc7, 0x0b, 0x4f, 0x1d,
    0x8a, 0x51, 0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31, 0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64,
    0xea, 0xc5, 0xac, 0x83, 0x34, 0xd3, 0xeb, 0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb,
    0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0, 0xda, 0x49, 0xd3, 0x16, 0x55, 0x26, 0x29, 0xd4, 0x68, 0x9e,
    0x2b, 0x16, 0xbe, 0x58, 0x7d, 0x47, 0xa1, 0xfc, 0x8f, 0xf8, 0xb8, 0xd1, 0x7a, 0xd0, 0x31, 0xce,
    0x45, 0xcb, 0x3a, 0x8f, 0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b, 0x40, 0x7e,
};

#define P32_1 0x9E3779B1U
#define P32_2 0x85EBCA77U
#define P32_3 0xC2B2AE3DU
#define P64_1 0x9E3779B185EBCA87ULL
#define P64_2 0xC2B2AE3D27D4EB4FULL
#define P64_3 0x165667B19E3779F9ULL
#define P64_4 0x85EBCA77C2B2AE63ULL
#define P64_5 0x27D4EB2F165667C5ULL
#define PMX1 0x165667919E3779F9ULL
#define PMX2 0x9FB21C651E98DF25ULL

static uint64_t rd64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
    return v;
}
static uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static uint32_t swap32(uint32_t x) {
    return ((x << 24) & 0xff000000U) | ((x << 8) & 0x00ff0000U) | ((x >> 8) & 0x0000ff00U) |
           ((x >> 24) & 0x000000ffU);
}
static uint64_t swap64(uint64_t x) {
    return ((uint64_t)swap32((uint32_t)x) << 32) | swap32((uint32_t)(x >> 32));
}
static uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

static void mul128(uint64_t a, uint64_t b, uint64_t* lo, uint64_t* hi) {
    unsigned __int128 p = (unsigned __int128)a * b;
    *lo = (uint64_t)p;
    *hi = (uint64_t)(p >> 64);
}
static uint64_t mul_fold64(uint64_t a, uint64_t b) {
    uint64_t lo, hi;
    mul128(a, b, &lo, &hi);
    return lo ^ hi;
}
static uint64_t xxh64_avalanche(uint64_t h) {
    h ^= h >> 33;
    h *= P64_2;
    h ^= h >> 29;
    h *= P64_3;
    h ^= h >> 32;
    return h;
}
static uint64_t xxh3_avalanche(uint64_t h) {
    h ^= h >> 37;
    h *= PMX1;
    h ^= h >> 32;
    return h;
}
static uint64_t rrmxmx(uint64_t h, uint64_t len) {
    h ^= rotl64(h, 49) ^ rotl64(h, 24);
    h *= PMX2;
    h ^= (h >> 35) + len;
    h *= PMX2;
    return h ^ (h >> 28);
}
static uint64_t mix16(const uint8_t* in, const uint8_t* sec, uint64_t seed) {
    return mul_fold64(rd64(in) ^ (rd64(sec) + seed), rd64(in + 8) ^ (rd64(sec + 8) - seed));
}

/* long-input accumulation (> 240 B): stripes of 64 B, 16 stripes per 1 KiB block */
__attribute__((unused)) static void accumulate_512(uint64_t acc[8], const uint8_t* in, const uint8_t* sec) {
    for (int i = 0; i < 8; ++i) {
        uint64_t v = rd64(in + 8 * i);
        uint64_t k = v ^ rd64(sec + 8 * i);
        acc[i ^ 1] += v;
        acc[i] += (uint64_t)(uint32_t)k * (k >> 32);
    }
}
__attribute__((unused)) static void scramble(uint64_t acc[8], const uint8_t* sec) {
    for (int i = 0; i < 8; ++i) {
        uint64_t a = acc[i];
        a ^= a >> 47;
        a ^= rd64(sec + 8 * i);
        a *= P32_1;
        acc[i] = a;
    }
}
#ifdef __AVX2__
/* The same two steps on 4 accumulators per 256-bit vector: XXH3's published
 * AVX2 kernels (the SIMD path xxhash-rust takes), so the cpu_baseline leg is
 * not handicapped by a scalar hash.  Identical results (tests/test_oracle.py KATs). */
#define accumulate_512 accumulate_512_avx2
#define scramble scramble_avx2
static void accumulate_512_avx2(uint64_t acc[8], const uint8_t* in, const uint8_t* sec) {
    for (int i = 0; i < 2; ++i) {
        __m256i a = _mm256_loadu_si256((const __m256i*)(acc + 4 * i));
        const __m256i d = _mm256_loadu_si256((const __m256i*)(in + 32 * i));
        const __m256i k = _mm256_xor_si256(d, _mm256_loadu_si256((const __m256i*)(sec + 32 * i)));
        const __m256i prod = _mm256_mul_epu32(k, _mm256_shuffle_epi32(k, _MM_SHUFFLE(0, 3, 0, 1)));
        a = _mm256_add_epi64(a, _mm256_shuffle_epi32(d, _MM_SHUFFLE(1, 0, 3, 2)));
        _mm256_storeu_si256((__m256i*)(acc + 4 * i), _mm256_add_epi64(a, prod));
    }
}
static void scramble_avx2(uint64_t acc[8], const uint8_t* sec) {
    const __m256i prime = _mm256_set1_epi32((int)P32_1);
    for (int i = 0; i < 2; ++i) {
        __m256i a = _mm256_loadu_si256((const __m256i*)(acc + 4 * i));
        a = _mm256_xor_si256(a, _mm256_srli_epi64(a, 47));
        a = _mm256_xor_si256(a, _mm256_loadu_si256((const __m256i*)(sec + 32 * i)));
        const __m256i lo = _mm256_mul_epu32(a, prime);
        const __m256i hi = _mm256_mul_epu32(_mm256_shuffle_epi32(a, _MM_SHUFFLE(0, 3, 0, 1)), prime);
        _mm256_storeu_si256((__m256i*)(acc + 4 * i), _mm256_add_epi64(lo, _mm256_slli_epi64(hi, 32)));
    }
}
#endif
static void hash_long(uint64_t acc[8], const uint8_t* in, size_t len) {
    const size_t stripes_per_block = (192 - 64) / 8; /* 16 */
    const size_t block_len = 64 * stripes_per_block; /* 1024 */
    const size_t nb_blocks = (len - 1) / block_len;
    acc[0] = P32_3; acc[1] = P64_1; acc[2] = P64_2; acc[3] = P64_3;
    acc[4] = P64_4; acc[5] = P32_2; acc[6] = P64_5; acc[7] = P32_1;
    for (size_t n = 0; n < nb_blocks; ++n) {
        for (size_t s = 0; s < stripes_per_block; ++s)
            accumulate_512(acc, in + n * block_len + s * 64, kSecret + s * 8);
        scramble(acc, kSecret + 192 - 64);
    }
    size_t nb_stripes = ((len - 1) - block_len * nb_blocks) / 64;
    for (size_t s = 0; s < nb_stripes; ++s)
        accumulate_512(acc, in + nb_blocks * block_len + s * 64, kSecret + s * 8);
    accumulate_512(acc, in + len - 64, kSecret + 192 - 64 - 7);
}
static uint64_t merge_accs(const uint64_t acc[8], const uint8_t* sec, uint64_t start) {
    uint64_t r = start;
    for (int i = 0; i < 4; ++i)
        r += mul_fold64(acc[2 * i] ^ rd64(sec + 16 * i), acc[2 * i + 1] ^ rd64(sec + 16 * i + 8));
    return xxh3_avalanche(r);
}

uint64_t orc_xxh3_64(const uint8_t* p, size_t len) {
    const uint8_t* s = kSecret;
    if (len == 0) return xxh64_avalanche(rd64(s + 56) ^ rd64(s + 64));
    if (len <= 3) {
        uint32_t c1 = p[0], c2 = p[len >> 1], c3 = p[len - 1];
        uint32_t combined = (c1 << 16) | (c2 << 24) | c3 | ((uint32_t)len << 8);
        uint64_t bitflip = (uint64_t)(rd32(s) ^ rd32(s + 4));
        return xxh64_avalanche((uint64_t)combined ^ bitflip);
    }
    if (len <= 8) {
        uint32_t in1 = rd32(p), in2 = rd32(p + len - 4);
        uint64_t bitflip = rd64(s + 8) ^ rd64(s + 16);
        uint64_t in64 = in2 + ((uint64_t)in1 << 32);
        return rrmxmx(in64 ^ bitflip, len);
    }
    if (len <= 16) {
        uint64_t bf1 = rd64(s + 24) ^ rd64(s + 32);
        uint64_t bf2 = rd64(s + 40) ^ rd64(s + 48);
        uint64_t lo = rd64(p) ^ bf1;
        uint64_t hi = rd64(p + len - 8) ^ bf2;
        uint64_t acc = len + swap64(lo) + hi + mul_fold64(lo, hi);
        return xxh3_avalanche(acc);
    }
    if (len <= 128) {
        uint64_t acc = len * P64_1;
        if (len > 32) {
            if (len > 64) {
                if (len > 96) {
                    acc += mix16(p + 48, s + 96, 0);
                    acc += mix16(p + len - 64, s + 112, 0);
                }
                acc += mix16(p + 32, s + 64, 0);
                acc += mix16(p + len - 48, s + 80, 0);
            }
            acc += mix16(p + 16, s + 32, 0);
            acc += mix16(p + len - 32, s + 48, 0);
        }
        acc += mix16(p, s, 0);
        acc += mix16(p + len - 16, s + 16, 0);
        return xxh3_avalanche(acc);
    }
    if (len <= 240) {
        uint64_t acc = len * P64_1;
        size_t rounds = len / 16;
        for (size_t i = 0; i < 8; ++i) acc += mix16(p + 16 * i, s + 16 * i, 0);
        acc = xxh3_avalanche(acc);
        for (size_t i = 8; i < rounds; ++i) acc += mix16(p + 16 * i, s + 16 * (i - 8) + 3, 0);
        acc += mix16(p + len - 16, s + 136 - 17, 0);
        return xxh3_avalanche(acc);
    }
    uint64_t acc[8];
    hash_long(acc, p, len);
    return merge_accs(acc, s + 11, (uint64_t)len * P64_1);
}

static void mix32(uint64_t* lo, uint64_t* hi, const uint8_t* in1, const uint8_t* in2,
                  const uint8_t* sec, uint64_t seed) {
    *lo += mix16(in1, sec, seed);
    *lo ^= rd64(in2) + rd64(in2 + 8);
    *hi += mix16(in2, sec + 16, seed);
    *hi ^= rd64(in1) + rd64(in1 + 8);
}

void orc_xxh3_128(const uint8_t* p, size_t len, uint64_t* out_lo, uint64_t* out_hi) {
    const uint8_t* s = kSecret;
    if (len == 0) {
        *out_lo = xxh64_avalanche(rd64(s + 64) ^ rd64(s + 72));
        *out_hi = xxh64_avalanche(rd64(s + 80) ^ rd64(s + 88));
        return;
    }
    if (len <= 3) {
        uint32_t c1 = p[0], c2 = p[len >> 1], c3 = p[len - 1];
        uint32_t cl = (c1 << 16) | (c2 << 24) | c3 | ((uint32_t)len << 8);
        uint32_t ch = rotl32(swap32(cl), 13);
        uint64_t bfl = (uint64_t)(rd32(s) ^ rd32(s + 4));
        uint64_t bfh = (uint64_t)(rd32(s + 8) ^ rd32(s + 12));
        *out_lo = xxh64_avalanche((uint64_t)cl ^ bfl);
        *out_hi = xxh64_avalanche((uint64_t)ch ^ bfh);
        return;
    }
    if (len <= 8) {
        uint32_t in_lo = rd32(p), in_hi = rd32(p + len - 4);
        uint64_t in64 = in_lo + ((uint64_t)in_hi << 32);
        uint64_t bitflip = rd64(s + 16) ^ rd64(s + 24);
        uint64_t keyed = in64 ^ bitflip;
        uint64_t lo, hi;
        mul128(keyed, P64_1 + ((uint64_t)len << 2), &lo, &hi);
        hi += lo << 1;
        lo ^= hi >> 3;
        lo ^= lo >> 35;
        lo *= PMX2;
        lo ^= lo >> 28;
        hi = xxh3_avalanche(hi);
        *out_lo = lo;
        *out_hi = hi;
        return;
    }
    if (len <= 16) {
        uint64_t bfl = rd64(s + 32) ^ rd64(s + 40);
        uint64_t bfh = rd64(s + 48) ^ rd64(s + 56);
        uint64_t in_lo = rd64(p);
        uint64_t in_hi = rd64(p + len - 8);
        uint64_t mlo, mhi;
        mul128(in_lo ^ in_hi ^ bfl, P64_1, &mlo, &mhi);
        mlo += (uint64_t)(len - 1) << 54;
        in_hi ^= bfh;
        mhi += in_hi + (uint64_t)(uint32_t)in_hi * (uint64_t)(P32_2 - 1);
        mlo ^= swap64(mhi);
        uint64_t hlo, hhi;
        mul128(mlo, P64_2, &hlo, &hhi);
        hhi += mhi * P64_2;
        *out_lo = xxh3_avalanche(hlo);
        *out_hi = xxh3_avalanche(hhi);
        return;
    }
    uint64_t alo, ahi;
    if (len <= 128) {
        alo = len * P64_1;
        ahi = 0;
        if (len > 32) {
            if (len > 64) {
                if (len > 96) mix32(&alo, &ahi, p + 48, p + len - 64, s + 96, 0);
                mix32(&alo, &ahi, p + 32, p + len - 48, s + 64, 0);
            }
            mix32(&alo, &ahi, p + 16, p + len - 32, s + 32, 0);
        }
        mix32(&alo, &ahi, p, p + len - 16, s, 0);
    } else if (len <= 240) {
        alo = len * P64_1;
        ahi = 0;
        for (size_t i = 32; i < 160; i += 32) mix32(&alo, &ahi, p + i - 32, p + i - 16, s + i - 32, 0);
        alo = xxh3_avalanche(alo);
        ahi = xxh3_avalanche(ahi);
        for (size_t i = 160; i <= len; i += 32)
            mix32(&alo, &ahi, p + i - 32, p + i - 16, s + 3 + i - 160, 0);
        mix32(&alo, &ahi, p + len - 16, p + len - 32, s + 136 - 17 - 16, 0);
    } else {
        uint64_t acc[8];
        hash_long(acc, p, len);
        *out_lo = merge_accs(acc, s + 11, (uint64_t)len * P64_1);
        *out_hi = merge_accs(acc, s + 192 - 64 - 11, ~((uint64_t)len * P64_2));
        return;
    }
    uint64_t hlo = alo + ahi;
    uint64_t hhi = alo * P64_1 + ahi * P64_4 + (uint64_t)len * P64_2;
    *out_lo = xxh3_avalanche(hlo);
    *out_hi = 0 - xxh3_avalanche(hhi);
}
