/*
 * fuzz_driver.c — TEST INFRASTRUCTURE ONLY: a seeded property / mutation run
 * of the oracle for the host sanitizer build (make -C oracle asan; run by
 * tests/test_oracle.py::test_oracle_asan, SURVEY.md §5 "run the C++ oracle
 * under ASan/UBSan on the host").  Properties after fuzz/data_block's harness
 * (fuzz/data_block/src/main.rs:130-323): random sorted, deduplicated items
 * (MVCC versions of one key, tombstones, empty values, 1..10-byte seqnos),
 * restart interval 1..255, hash ratio in [0, 8): encode -> verify -> decode
 * round trip, every point_read; then byte flips of the payload re-sealed with a
 * valid checksum (the decoder must report, never read out of bounds), random
 * LZ4 streams, and every XXH3 length class.  Exit status 0 = all properties
 * held and the sanitizers stayed quiet.
 */
#include "lsm_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t rng_state;
static uint64_t rnd(void) { /* splitmix64 */
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static uint64_t rn(uint64_t n) { return n ? rnd() % n : 0; }

#define FAIL(...) do { fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); return 1; } while (0)

static int cmp_key(const uint8_t* a, size_t al, const uint8_t* b, size_t bl) {
    int c = memcmp(a, b, al < bl ? al : bl);
    return c ? c : (al < bl ? -1 : al > bl);
}

static int one_case(int iter) {
    const uint64_t n = 1 + rn(iter % 7 == 0 ? 600 : 80);
    uint8_t* keys = malloc(n * 40 + 1);
    uint8_t* vals = malloc(n * 300 + 1);
    uint64_t* ko = malloc((n + 1) * 8);
    uint64_t* vo = malloc((n + 1) * 8);
    uint64_t* seq = malloc(n * 8);
    uint8_t* vt = malloc(n);
    /* sorted keys: a random common prefix, a counter, random tails; MVCC runs share a key
     * with descending seqnos (key.rs:265-269) */
    const size_t pre = rn(24);
    uint8_t prefix[24];
    for (size_t i = 0; i < pre; ++i) prefix[i] = (uint8_t)rnd();
    size_t kp = 0, vp = 0;
    ko[0] = vo[0] = 0;
    uint64_t i = 0;
    while (i < n) {
        const uint64_t versions = (rn(5) == 0) ? 1 + rn(4) : 1;
        const size_t tail = rn(8);
        uint64_t s = rn(4) == 0 ? rnd() : rn(1 << 20) + versions;
        for (uint64_t v = 0; v < versions && i < n; ++v, ++i) {
            memcpy(keys + kp, prefix, pre);
            const uint32_t c = (uint32_t)(i - v);
            keys[kp + pre] = (uint8_t)(c >> 24); keys[kp + pre + 1] = (uint8_t)(c >> 16);
            keys[kp + pre + 2] = (uint8_t)(c >> 8); keys[kp + pre + 3] = (uint8_t)c;
            for (size_t t = 0; t < tail; ++t) keys[kp + pre + 4 + t] = (uint8_t)(c * 31 + t);
            kp += pre + 4 + tail;
            ko[i + 1] = kp;
            const uint64_t r = rn(10);
            vt[i] = r == 0 ? 1 : r == 1 ? 2 : r == 2 ? 4 : 0;
            const size_t vl = (vt[i] == 1 || vt[i] == 2) ? 0 : rn(rn(6) == 0 ? 300 : 40);
            for (size_t t = 0; t < vl; ++t) vals[vp + t] = (uint8_t)rnd();
            vp += vl;
            vo[i + 1] = vp;
            seq[i] = s - v;
        }
    }
    orc_items it = {keys, ko, vals, vo, seq, vt, NULL, NULL, n};
    const uint8_t ri = (uint8_t)(rn(3) == 0 ? 1 + rn(255) : 1 + rn(16));
    const float ratio = rn(3) == 0 ? 0.0f : (float)rn(800) / 100.0f;
    const size_t cap = 64 + kp + vp + 40 * n + 8 * n + (size_t)(ratio * n) + 4096;
    uint8_t* pay = malloc(cap);
    int64_t plen = orc_data_block_encode(&it, 0, n, ri, ratio, pay, cap);
    if (plen < 0) FAIL("iter %d: encode status %lld", iter, (long long)-plen);
    uint8_t* blk = malloc((size_t)plen + 33);
    if (orc_block_write(pay, (size_t)plen, 0, blk, (size_t)plen + 33) != plen + 33) FAIL("iter %d: write", iter);
    orc_header h;
    if (orc_block_verify(blk, (size_t)plen + 33, &h) != ORC_OK) FAIL("iter %d: verify", iter);
    uint64_t* psq = malloc(n * 8); uint32_t* pko = malloc(n * 4); uint32_t* pvo = malloc(n * 4);
    uint32_t* pvl = malloc(n * 4); uint16_t* pkl = malloc(n * 2); uint16_t* ppl = malloc(n * 2);
    uint8_t* pvt = malloc(n); uint64_t* pho = malloc(n * 8);
    orc_parsed o = {psq, pko, pvo, pvl, pkl, ppl, pvt, pho};
    const int64_t got = orc_data_block_decode(pay, (size_t)plen, &o, 0, n);
    if (got != (int64_t)n) FAIL("iter %d: decode %lld of %llu", iter, (long long)got, (unsigned long long)n);
    uint8_t key[128];
    for (uint64_t j = 0; j < n; ++j) {  /* materialize == input (data_block/mod.rs:296-315) */
        const uint64_t hd = (j / ri) * ri;
        memcpy(key, pay + pko[hd], ppl[j]);
        memcpy(key + ppl[j], pay + pko[j], pkl[j]);
        const size_t kl = (size_t)ppl[j] + pkl[j];
        if (kl != ko[j + 1] - ko[j] || memcmp(key, keys + ko[j], kl)) FAIL("iter %d: key %llu", iter, (unsigned long long)j);
        if (psq[j] != seq[j] || pvt[j] != vt[j]) FAIL("iter %d: fields %llu", iter, (unsigned long long)j);
        if (vt[j] != 1 && vt[j] != 2 && (pvl[j] != vo[j + 1] - vo[j] || memcmp(pay + pvo[j], vals + vo[j], pvl[j])))
            FAIL("iter %d: value %llu", iter, (unsigned long long)j);
    }
    for (uint64_t j = 0; j < n; ++j) {  /* point_read: newest version with seqno < snapshot */
        const uint8_t* kj = keys + ko[j];
        const size_t kl = ko[j + 1] - ko[j];
        const uint64_t snap = seq[j] + 1;
        int64_t want = -1;
        for (uint64_t q = 0; q < n; ++q)
            if (!cmp_key(keys + ko[q], ko[q + 1] - ko[q], kj, kl) && seq[q] < snap) { want = (int64_t)q; break; }
        const int64_t pr = orc_data_block_point_read(pay, (size_t)plen, kj, kl, snap);
        if (pr != want) FAIL("iter %d: point_read %llu got %lld want %lld", iter, (unsigned long long)j, (long long)pr, (long long)want);
    }
    /* mutations: flip bytes, re-seal, decode must report or succeed within bounds */
    uint8_t* mut = malloc((size_t)plen + 64);
    for (int m = 0; m < 24; ++m) {
        memcpy(mut, pay, (size_t)plen);
        const int flips = 1 + (int)rn(4);
        for (int f = 0; f < flips; ++f) mut[rn((uint64_t)plen)] ^= (uint8_t)(1 + rn(255));
        (void)orc_data_block_decode(mut, (size_t)plen, &o, 0, n);
        (void)orc_data_block_point_read(mut, (size_t)plen, keys, ko[1], ~0ULL >> 1);
        uint8_t* blk2 = malloc((size_t)plen + 33);
        orc_block_write(mut, (size_t)plen, 0, blk2, (size_t)plen + 33);
        blk2[rn((uint64_t)plen + 33)] ^= (uint8_t)(1 + rn(255));
        (void)orc_block_verify(blk2, (size_t)plen + 33, &h);
        (void)orc_block_verify(blk2, rn((uint64_t)plen + 34), &h);  /* truncated handles */
        free(blk2);
    }
    free(mut);
    free(psq); free(pko); free(pvo); free(pvl); free(pkl); free(ppl); free(pvt); free(pho);
    free(blk); free(pay); free(keys); free(vals); free(ko); free(vo); free(seq); free(vt);
    return 0;
}

int main(int argc, char** argv) {
    rng_state = argc > 1 ? strtoull(argv[1], NULL, 0) : 0x5EED;
    const int iters = argc > 2 ? atoi(argv[2]) : 300;
    for (int i = 0; i < iters; ++i)
        if (one_case(i)) return 1;
    /* XXH3 every length class, LZ4 random streams */
    uint8_t buf[4096], out[8192];
    for (size_t len = 0; len < sizeof buf; len += 1 + (len > 300 ? 37 : 0)) {
        for (size_t k = 0; k < len; ++k) buf[k] = (uint8_t)rnd();
        uint64_t lo, hi;
        orc_xxh3_128(len ? buf : NULL, len, &lo, &hi);
        (void)orc_xxh3_64(len ? buf : NULL, len);
    }
    for (int i = 0; i < 2000; ++i) {
        const size_t len = rn(300);
        for (size_t k = 0; k < len; ++k) buf[k] = (uint8_t)(rn(4) ? rnd() : rn(16));
        (void)orc_lz4_decompress(buf, len, out, rn(sizeof out));
    }
    printf("fuzz_driver ok: %d cases\n", iters);
    return 0;
}
