/*
 * batch.c — TEST INFRASTRUCTURE ONLY (see lsm_oracle.h).
 *
 * Batched CPU path over many blocks, split into contiguous block ranges per
 * pthread.  Per block it does exactly what the reference does per call:
 *   encode: DataBlock::encode_into into a scratch Vec, then Block::write_into
 *           the output (src/table/writer/mod.rs:303-322)
 *   decode: Block::from_file (header + xxh3_128 verify) then the full forward
 *           DataBlock::iter() (src/table/block/mod.rs:131-182, decoder.rs:442)
 * This is the bench.py `cpu_baseline` ("port") and the parity checker.
 */
#include "lsm_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define HDR_LEN 33

typedef struct enc_job {
    const orc_items* it;
    const uint32_t* starts;
    uint32_t b0, b1;
    uint8_t ri, type;
    float ratio;
    uint8_t* buf;     /* thread-local output (headers + payloads) */
    size_t len, cap;
    uint64_t* sizes;  /* per block on-disk size, indexed by block */
    int status;
} enc_job;

static void* enc_worker(void* arg) {
    enc_job* j = (enc_job*)arg;
    size_t scratch_cap = 1 << 16;
    uint8_t* scratch = (uint8_t*)malloc(scratch_cap);
    for (uint32_t b = j->b0; b < j->b1 && !j->status; ++b) {
        uint64_t first = j->starts[b], count = j->starts[b + 1] - j->starts[b];
        int64_t n;
        for (;;) {
            n = (j->type == 1) ? orc_index_block_encode(j->it, first, count, scratch, scratch_cap)
                               : orc_data_block_encode(j->it, first, count, j->ri, j->ratio, scratch,
                                                       scratch_cap);
            if (n != -ORC_OVERFLOW) break;
            scratch_cap *= 2;
            scratch = (uint8_t*)realloc(scratch, scratch_cap);
        }
        if (n < 0) { j->status = (int)-n; break; }
        if (j->len + HDR_LEN + (size_t)n > j->cap) {
            while (j->len + HDR_LEN + (size_t)n > j->cap) j->cap = j->cap * 2 + 4096;
            j->buf = (uint8_t*)realloc(j->buf, j->cap);
        }
        int64_t w = orc_block_write(scratch, (size_t)n, j->type, j->buf + j->len, j->cap - j->len);
        if (w < 0) { j->status = (int)-w; break; }
        j->len += (size_t)w;
        j->sizes[b] = (uint64_t)w;
    }
    free(scratch);
    return NULL;
}

static int clamp_threads(int nthreads, uint32_t n) {
    if (nthreads < 1) nthreads = 1;
    if ((uint32_t)nthreads > n) nthreads = n ? (int)n : 1;
    return nthreads;
}

int orc_encode_blocks(const orc_items* it, const uint32_t* starts, uint32_t n_blocks, uint8_t ri,
                      float ratio, uint8_t type, uint8_t* out, uint64_t cap, uint64_t* block_off,
                      int nthreads) {
    nthreads = clamp_threads(nthreads, n_blocks);
    enc_job* jobs = (enc_job*)calloc((size_t)nthreads, sizeof(enc_job));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    uint64_t* sizes = (uint64_t*)calloc((size_t)n_blocks + 1, sizeof(uint64_t));
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].it = it; jobs[t].starts = starts;
        jobs[t].b0 = (uint32_t)((uint64_t)n_blocks * t / nthreads);
        jobs[t].b1 = (uint32_t)((uint64_t)n_blocks * (t + 1) / nthreads);
        jobs[t].ri = ri; jobs[t].type = type; jobs[t].ratio = ratio;
        jobs[t].cap = 1 << 20;
        jobs[t].buf = (uint8_t*)malloc(jobs[t].cap);
        jobs[t].sizes = sizes;
        pthread_create(&th[t], NULL, enc_worker, &jobs[t]);
    }
    int status = 0;
    for (int t = 0; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
        if (jobs[t].status && !status) status = jobs[t].status;
    }
    if (!status) {
        block_off[0] = 0;
        for (uint32_t b = 0; b < n_blocks; ++b) block_off[b + 1] = block_off[b] + sizes[b];
        if (block_off[n_blocks] > cap) status = ORC_OVERFLOW;
    }
    if (!status)
        for (int t = 0; t < nthreads; ++t)
            if (jobs[t].b1 > jobs[t].b0) memcpy(out + block_off[jobs[t].b0], jobs[t].buf, jobs[t].len);
    for (int t = 0; t < nthreads; ++t) free(jobs[t].buf);
    free(jobs); free(th); free(sizes);
    return status ? -status : 0;
}

typedef struct dec_job {
    const uint8_t* blocks;
    const uint64_t* off;
    uint32_t b0, b1;
    int expect_type;
    orc_parsed* out;
    const uint32_t* item_start;
    int32_t* status;
    uint64_t fold;
    uint64_t items;
    int materialize;
} dec_job;

static int decode_one(const uint8_t* blk, size_t len, int expect_type, orc_parsed* out,
                      uint64_t base, uint64_t cap, uint64_t* nitems) {
    orc_header h;
    int st = orc_block_verify(blk, len, &h);
    if (st) return st;
    if (expect_type >= 0 && h.block_type != (uint8_t)expect_type) return ORC_TYPE_MISMATCH;  /* util.rs:81-86 */
    int64_t n;
    if (h.block_type == 0 || h.block_type == 3) n = orc_data_block_decode(blk + HDR_LEN, len - HDR_LEN, out, base, cap);
    else if (h.block_type == 1) n = orc_index_block_decode(blk + HDR_LEN, len - HDR_LEN, out, base, cap);
    else return ORC_UNSUPPORTED;
    if (n < 0) return (int)-n;
    *nitems = (uint64_t)n;
    return ORC_OK;
}

static void* dec_worker(void* arg) {
    dec_job* j = (dec_job*)arg;
    for (uint32_t b = j->b0; b < j->b1; ++b) {
        uint64_t base = j->item_start[b], cap = j->item_start[b + 1] - base, n = 0;
        int st = decode_one(j->blocks + j->off[b], (size_t)(j->off[b + 1] - j->off[b]), j->expect_type,
                            j->out, base, cap, &n);
        j->status[b] = st;
        j->items += n;
    }
    return NULL;
}

int orc_decode_blocks(const uint8_t* blocks, const uint64_t* off, uint32_t n_blocks, int expect_type,
                      orc_parsed* out, uint64_t item_cap, uint32_t* item_start, int32_t* status,
                      int nthreads) {
    /* item_start from the trailers' item_count (trailer.rs:57-75) */
    item_start[0] = 0;
    uint64_t acc = 0;
    for (uint32_t b = 0; b < n_blocks; ++b) {
        size_t len = (size_t)(off[b + 1] - off[b]);
        uint32_t c = 0;
        if (len >= HDR_LEN && orc_trailer_item_count(blocks + off[b] + HDR_LEN, len - HDR_LEN, &c) == ORC_OK) {
            /* a record is >= 3 bytes, so an unverified trailer may claim at most
             * (payload - 32) / 3 items: bounds what a corrupt block can reserve */
            uint64_t most = (uint64_t)(len - HDR_LEN - 32) / 3;
            acc += c < most ? c : most;
        }
        if (acc > item_cap) acc = item_cap;
        item_start[b + 1] = (uint32_t)acc;
    }
    nthreads = clamp_threads(nthreads, n_blocks);
    dec_job* jobs = (dec_job*)calloc((size_t)nthreads, sizeof(dec_job));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].blocks = blocks; jobs[t].off = off;
        jobs[t].b0 = (uint32_t)((uint64_t)n_blocks * t / nthreads);
        jobs[t].b1 = (uint32_t)((uint64_t)n_blocks * (t + 1) / nthreads);
        jobs[t].expect_type = expect_type; jobs[t].out = out;
        jobs[t].item_start = item_start; jobs[t].status = status;
        pthread_create(&th[t], NULL, dec_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    free(jobs); free(th);
    return 0;
}

/* decode + materialize (Slice::fused(prefix, suffix), data_block/mod.rs:296-315)
 * with per-thread scratch; folds key bytes so nothing is elided. */
static void* mat_worker(void* arg) {
    dec_job* j = (dec_job*)arg;
    size_t cap = 4096;
    uint64_t* sq = (uint64_t*)malloc(8 * cap);
    uint32_t* ko = (uint32_t*)malloc(4 * cap);
    uint32_t* vo = (uint32_t*)malloc(4 * cap);
    uint32_t* vl = (uint32_t*)malloc(4 * cap);
    uint16_t* kl = (uint16_t*)malloc(2 * cap);
    uint16_t* pl = (uint16_t*)malloc(2 * cap);
    uint8_t* vt = (uint8_t*)malloc(cap);
    uint8_t key[65536 * 2];
    for (uint32_t b = j->b0; b < j->b1; ++b) {
        const uint8_t* blk = j->blocks + j->off[b];
        size_t len = (size_t)(j->off[b + 1] - j->off[b]);
        uint32_t c = 0;
        if (len < HDR_LEN || orc_trailer_item_count(blk + HDR_LEN, len - HDR_LEN, &c)) continue;
        if (c > cap) {
            while (c > cap) cap *= 2;
            sq = realloc(sq, 8 * cap); ko = realloc(ko, 4 * cap); vo = realloc(vo, 4 * cap);
            vl = realloc(vl, 4 * cap); kl = realloc(kl, 2 * cap); pl = realloc(pl, 2 * cap); vt = realloc(vt, cap);
        }
        orc_parsed o = {sq, ko, vo, vl, kl, pl, vt, NULL};
        uint64_t n = 0;
        if (decode_one(blk, len, -1, &o, 0, cap, &n)) continue;
        const uint8_t* pay = blk + HDR_LEN;
        uint32_t ri = pay[len - HDR_LEN - 31];
        for (uint64_t i = 0; i < n; ++i) {
            uint64_t h = (i / ri) * ri;
            memcpy(key, pay + ko[h], pl[i]);
            memcpy(key + pl[i], pay + ko[i], kl[i]);
            size_t klen = (size_t)pl[i] + kl[i];
            uint64_t f = klen ^ sq[i] ^ ((uint64_t)vl[i] << 20) ^ vo[i];
            if (klen >= 8) { uint64_t w; memcpy(&w, key + klen - 8, 8); f ^= w; }
            j->fold = j->fold * 0x100000001B3ULL + f;
        }
        j->items += n;
    }
    free(sq); free(ko); free(vo); free(vl); free(kl); free(pl); free(vt);
    return NULL;
}

uint64_t orc_decode_materialize_blocks(const uint8_t* blocks, const uint64_t* off, uint32_t n_blocks,
                                       int nthreads, uint64_t* fold) {
    nthreads = clamp_threads(nthreads, n_blocks);
    dec_job* jobs = (dec_job*)calloc((size_t)nthreads, sizeof(dec_job));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].blocks = blocks; jobs[t].off = off;
        jobs[t].b0 = (uint32_t)((uint64_t)n_blocks * t / nthreads);
        jobs[t].b1 = (uint32_t)((uint64_t)n_blocks * (t + 1) / nthreads);
        pthread_create(&th[t], NULL, mat_worker, &jobs[t]);
    }
    uint64_t items = 0, f = 0;
    for (int t = 0; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
        items += jobs[t].items;
        f ^= jobs[t].fold;
    }
    if (fold) *fold = f;
    free(jobs); free(th);
    return items;
}
