/*
 * block.c — TEST INFRASTRUCTURE ONLY (see lsm_oracle.h).
 *
 * Scalar restatement of the fjall-rs/lsm-tree 3.1.9 v3 block format:
 *   Block header                src/table/block/header.rs:49-169
 *   Block::write_into/from_file src/table/block/mod.rs:45-182
 *   Encoder                     src/table/block/encoder.rs:84-164
 *   Trailer                     src/table/block/trailer.rs:12-174
 *   binary index                src/table/block/binary_index/{builder,reader}.rs
 *   hash index                  src/table/block/hash_index/{mod,builder,reader}.rs
 *   DataBlock record format     src/table/data_block/mod.rs:27-264
 *   Decoder::next               src/table/block/decoder.rs:442-483
 *   IndexBlock records          src/table/index_block/block_handle.rs:134-206
 *   point_read                  src/table/data_block/mod.rs:412-472
 *   Writer chunking             src/table/writer/mod.rs:243-296
 *
 * Where the reference panics on malformed payload bytes (unwrap!/expect,
 * src/lib.rs:62-66) this restatement returns ORC_PARSE instead; on
 * well-formed blocks every output is identical.  The GPU decoder applies the
 * same validation rules (DESIGN.md "Decode validation").
 */
#include "lsm_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define HDR_LEN 33
#define TRAILER_LEN 31
#define TRAILER_MARKER 0xFF
#define HASH_FREE 254
#define HASH_CONFLICT 255
#define HASH_MAX_POINTERS 254

static void put32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}
static void put16(uint8_t* p, uint16_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); }
static void put64(uint8_t* p, uint64_t v) { for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (8 * i)); }
static uint32_t get32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static uint16_t get16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static uint64_t get64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
    return v;
}

size_t orc_varint_len(uint64_t v) {
    size_t n = 1;
    while (v >= 0x80) { v >>= 7; ++n; }
    return n;
}
/* varint-rs VarintWriter::write_*_varint: 7-bit groups, low first, MSB = more */
size_t orc_varint_put(uint8_t* out, uint64_t v) {
    size_t n = 0;
    while (v >= 0x80) { out[n++] = (uint8_t)(v | 0x80); v >>= 7; }
    out[n++] = (uint8_t)v;
    return n;
}

/* Growable byte sink standing in for the reference's `&mut Vec<u8>`. */
typedef struct sink { uint8_t* p; size_t len, cap; int overflow; } sink;
static void s_put(sink* s, const void* src, size_t n) {
    if (s->len + n > s->cap) { s->overflow = 1; s->len += n; return; }
    memcpy(s->p + s->len, src, n);
    s->len += n;
}
static void s_u8(sink* s, uint8_t v) { s_put(s, &v, 1); }
static void s_var(sink* s, uint64_t v) { uint8_t b[10]; size_t n = orc_varint_put(b, v); s_put(s, b, n); }
static void s_u32(sink* s, uint32_t v) { uint8_t b[4]; put32(b, v); s_put(s, b, 4); }
static void s_u16(sink* s, uint16_t v) { uint8_t b[2]; put16(b, v); s_put(s, b, 2); }

static int is_tombstone(uint8_t vt) { return vt == 1 || vt == 2; }  /* value_type.rs:27-29 */
static int valid_vtype(uint8_t vt) { return vt == 0 || vt == 1 || vt == 2 || vt == 4; }

/* hash_index/builder.rs:39-63 — f32 multiply, saturating `as u32` */
static uint32_t bucket_count(uint64_t items, float ratio) {
    if (!(ratio > 0.0f)) return 0;
    float prod = (float)items * ratio;
    uint32_t b;
    if (isnan(prod) || prod <= 0.0f) b = 0;
    else if (prod >= 4294967296.0f) b = 0xFFFFFFFFu;
    else b = (uint32_t)prod;
    return b < 1 ? 1 : b;
}

/* util.rs:125-130 */
static size_t lcp(const uint8_t* a, size_t an, const uint8_t* b, size_t bn) {
    size_t n = an < bn ? an : bn, i = 0;
    while (i < n && a[i] == b[i]) ++i;
    return i;
}

/* Trailer::write (trailer.rs:78-173) + binary_index::Builder::write (builder.rs:19-54) */
static void write_trailer(sink* s, uint8_t ri, const uint32_t* bin, uint32_t bin_len,
                          const uint8_t* hash, uint32_t buckets, uint32_t item_count) {
    s_u8(s, TRAILER_MARKER);
    uint32_t bin_off = (uint32_t)s->len;
    uint8_t step = bin[bin_len - 1] <= 0xFFFF ? 2 : 4;
    for (uint32_t i = 0; i < bin_len; ++i) {
        if (step == 2) s_u16(s, (uint16_t)bin[i]); else s_u32(s, bin[i]);
    }
    uint32_t hash_off = 0;
    if (buckets > 0 && bin_len <= HASH_MAX_POINTERS) {
        hash_off = (uint32_t)s->len;
        s_put(s, hash, buckets);
    }
    s_u8(s, ri);
    s_u8(s, step);
    s_u32(s, bin_len);
    s_u32(s, bin_off);
    s_u32(s, hash_off > 0 ? buckets : 0);
    s_u32(s, hash_off);
    s_u8(s, 1);   /* prefix truncation on */
    s_u8(s, 0);   /* fixed key size (unused) */
    s_u16(s, 0);
    s_u8(s, 0);   /* fixed value size (unused) */
    s_u32(s, 0);
    s_u32(s, item_count);
}

/* hash_index::Builder::set (hash_index/builder.rs:64-110): FREE -> idx, same idx
 * -> kept, a different idx -> CONFLICT (sticky); bucket = hash64(key) % buckets
 * (hash_index/mod.rs:35-41). */
static void hash_set(uint8_t* hash, uint32_t buckets, const uint8_t* key, size_t klen, uint8_t idx) {
    uint32_t pos = (uint32_t)(orc_xxh3_64(key, klen) % buckets);
    uint8_t cur = hash[pos];
    if (cur == HASH_FREE) hash[pos] = idx;
    else if (cur != HASH_CONFLICT && cur != idx) hash[pos] = HASH_CONFLICT;
}

void orc_hash_index_build(const uint8_t* keys, const uint64_t* key_off, const uint8_t* idx, uint64_t n,
                          uint32_t buckets, uint8_t* out) {
    memset(out, HASH_FREE, buckets);              /* Builder::with_bucket_count, builder.rs:20-36 */
    for (uint64_t i = 0; i < n; ++i)
        hash_set(out, buckets, keys + key_off[i], (size_t)(key_off[i + 1] - key_off[i]), idx[i]);
}

uint8_t orc_hash_index_get(const uint8_t* bytes, uint32_t buckets, const uint8_t* key, size_t klen) {
    return bytes[orc_xxh3_64(key, klen) % buckets];  /* hash_index/reader.rs:46-58 */
}

int64_t orc_data_block_encode(const orc_items* it, uint64_t first, uint64_t count,
                              uint8_t ri, float ratio, uint8_t* out, size_t cap) {
    if (count == 0 || ri == 0 || signbit(ratio)) return -ORC_BAD_ARG; /* mod.rs:530, encoder.rs:91, builder.rs:40 */
    sink s = {out, 0, cap, 0};
    uint64_t n_restarts = (count + ri - 1) / ri;
    uint32_t* bin = (uint32_t*)malloc(sizeof(uint32_t) * n_restarts);
    uint32_t buckets = bucket_count(count, ratio);
    uint8_t* hash = (uint8_t*)malloc(buckets ? buckets : 1);
    memset(hash, HASH_FREE, buckets);
    uint32_t bin_len = 0;
    const uint8_t* base = NULL;
    size_t base_len = 0;
    for (uint64_t j = 0; j < count; ++j) {
        uint64_t i = first + j;
        const uint8_t* key = it->keys + it->key_off[i];
        size_t klen = (size_t)(it->key_off[i + 1] - it->key_off[i]);
        const uint8_t* val = it->vals + it->val_off[i];
        size_t vlen = (size_t)(it->val_off[i + 1] - it->val_off[i]);
        uint8_t vt = it->vtype[i];
        if (j % ri == 0) {
            bin[bin_len++] = (uint32_t)s.len;          /* encoder.rs:124-136 */
            s_u8(&s, vt);                              /* encode_full_into, mod.rs:195-219 */
            s_var(&s, it->seqno[i]);
            s_var(&s, (uint16_t)klen);
            s_put(&s, key, klen);
            base = key; base_len = klen;
        } else {
            size_t shared = lcp(base, base_len, key, klen);   /* encoder.rs:140-143 */
            s_u8(&s, vt);                              /* encode_truncated_into, mod.rs:221-264 */
            s_var(&s, it->seqno[i]);
            s_var(&s, (uint16_t)shared);
            s_var(&s, (uint16_t)(klen - shared));
            s_put(&s, key + shared, klen - shared);
        }
        if (!is_tombstone(vt)) {
            s_var(&s, (uint32_t)vlen);
            s_put(&s, val, vlen);
        }
        uint32_t restart_idx = bin_len - 1;
        if (buckets > 0 && restart_idx < HASH_MAX_POINTERS)  /* encoder.rs:148-154 */
            hash_set(hash, buckets, key, klen, (uint8_t)restart_idx);
    }
    write_trailer(&s, ri, bin, bin_len, hash, buckets, (uint32_t)count);
    free(bin);
    free(hash);
    if (s.overflow) return -ORC_OVERFLOW;
    return (int64_t)s.len;
}

int64_t orc_index_block_encode(const orc_items* it, uint64_t first, uint64_t count,
                               uint8_t* out, size_t cap) {
    if (count == 0) return -ORC_BAD_ARG;
    sink s = {out, 0, cap, 0};
    uint32_t* bin = (uint32_t*)malloc(sizeof(uint32_t) * count);
    for (uint64_t j = 0; j < count; ++j) {
        uint64_t i = first + j;
        size_t klen = (size_t)(it->key_off[i + 1] - it->key_off[i]);
        bin[j] = (uint32_t)s.len;
        s_u8(&s, 0);                         /* block_handle.rs:140 */
        s_var(&s, it->handle_off[i]);        /* BlockHandle::encode_into :45-50 */
        s_var(&s, it->handle_size[i]);
        s_var(&s, it->seqno[i]);
        s_var(&s, (uint16_t)klen);
        s_put(&s, it->keys + it->key_off[i], klen);
    }
    write_trailer(&s, 1, bin, (uint32_t)count, NULL, 0, (uint32_t)count);  /* index_block/mod.rs:117-118 */
    free(bin);
    if (s.overflow) return -ORC_OVERFLOW;
    return (int64_t)s.len;
}

int64_t orc_block_write(const uint8_t* payload, size_t len, uint8_t block_type, uint8_t* out,
                        size_t cap) {
    if (HDR_LEN + len > cap) return -ORC_OVERFLOW;
    if (block_type > 3) return -ORC_BAD_ARG;
    uint64_t lo, hi;
    orc_xxh3_128(payload, len, &lo, &hi);    /* block/mod.rs:70 */
    out[0] = 'L'; out[1] = 'S'; out[2] = 'M'; out[3] = 3;   /* file.rs:8 */
    out[4] = block_type;
    put64(out + 5, lo);
    put64(out + 13, hi);
    put32(out + 21, (uint32_t)len);
    put32(out + 25, (uint32_t)len);
    uint64_t hlo, hhi;
    orc_xxh3_128(out, 29, &hlo, &hhi);       /* header.rs:83-109 */
    put32(out + 29, (uint32_t)hlo);
    memmove(out + HDR_LEN, payload, len);
    return (int64_t)(HDR_LEN + len);
}

/* Header::encode_into (header.rs:80-112) of arbitrary field values. */
void orc_header_encode(uint8_t block_type, uint64_t ck_lo, uint64_t ck_hi, uint32_t data_length,
                       uint32_t uncompressed_length, uint8_t* out) {
    out[0] = 'L'; out[1] = 'S'; out[2] = 'M'; out[3] = 3;
    out[4] = block_type;
    put64(out + 5, ck_lo);
    put64(out + 13, ck_hi);
    put32(out + 21, data_length);
    put32(out + 25, uncompressed_length);
    uint64_t hlo, hhi;
    orc_xxh3_128(out, 29, &hlo, &hhi);
    put32(out + 29, (uint32_t)hlo);
}

int orc_header_decode(const uint8_t* buf, size_t len, orc_header* h) {
    if (len < 4) return ORC_TRUNCATED;
    if (!(buf[0] == 'L' && buf[1] == 'S' && buf[2] == 'M' && buf[3] == 3)) return ORC_BAD_MAGIC;
    if (len < 5) return ORC_TRUNCATED;
    if (buf[4] > 3) return ORC_BAD_TYPE;
    if (len < HDR_LEN) return ORC_TRUNCATED;
    uint64_t lo, hi;
    orc_xxh3_128(buf, 29, &lo, &hi);
    if ((uint32_t)lo != get32(buf + 29)) return ORC_HDR_CKSUM;
    h->block_type = buf[4];
    h->cksum_lo = get64(buf + 5);
    h->cksum_hi = get64(buf + 13);
    h->data_length = get32(buf + 21);
    h->uncompressed_length = get32(buf + 25);
    return ORC_OK;
}

int orc_block_verify(const uint8_t* buf, size_t len, orc_header* h) {
    int st = orc_header_decode(buf, len, h);
    if (st) return st;
    uint64_t lo, hi;
    orc_xxh3_128(buf + HDR_LEN, len - HDR_LEN, &lo, &hi);   /* block/mod.rs:141-149 */
    if (lo != h->cksum_lo || hi != h->cksum_hi) return ORC_CKSUM;
    if ((uint64_t)h->data_length != len - HDR_LEN) return ORC_TRUNCATED;
    return ORC_OK;
}

int orc_trailer_item_count(const uint8_t* payload, size_t len, uint32_t* count) {
    if (len < TRAILER_LEN + 1) return ORC_PARSE;
    *count = get32(payload + len - 4);
    return ORC_OK;
}

/* varint-rs VarintReader: value truncated to the type width (`as $type`),
 * more than max_bytes continuation bytes -> ORC_PARSE. */
static int rd_var(const uint8_t* p, size_t end, size_t* pos, int max_bytes, uint64_t mask,
                  uint64_t* v) {
    uint64_t acc = 0;
    for (int i = 0; i < max_bytes; ++i) {
        if (*pos >= end) return ORC_PARSE;
        uint8_t b = p[(*pos)++];
        acc |= (uint64_t)(b & 0x7F) << (7 * i);
        if (!(b & 0x80)) { *v = acc & mask; return ORC_OK; }
    }
    return ORC_PARSE;
}

typedef struct trailer_info {
    uint8_t ri, step;
    uint32_t bin_len, bin_off, hash_len, hash_off, item_count;
    size_t rec_end;  /* position of the 0xFF marker = bin_off - 1 */
} trailer_info;

static int read_trailer(const uint8_t* p, size_t len, trailer_info* t) {
    if (len < TRAILER_LEN + 1) return ORC_PARSE;
    const uint8_t* tr = p + len - TRAILER_LEN;   /* trailer.rs:29-33 */
    t->ri = tr[0];
    t->step = tr[1];
    t->bin_len = get32(tr + 2);
    t->bin_off = get32(tr + 6);
    t->hash_len = get32(tr + 10);
    t->hash_off = get32(tr + 14);
    t->item_count = get32(tr + 27);
    if (t->ri == 0 || (t->step != 2 && t->step != 4) || t->bin_len == 0 || t->bin_off == 0) return ORC_PARSE;
    if ((uint64_t)t->bin_off + (uint64_t)t->bin_len * t->step > len - TRAILER_LEN) return ORC_PARSE;
    if (p[t->bin_off - 1] != TRAILER_MARKER) return ORC_PARSE;
    if ((uint64_t)t->bin_len != ((uint64_t)t->item_count + t->ri - 1) / t->ri) return ORC_PARSE;
    t->rec_end = t->bin_off - 1;
    return ORC_OK;
}
static uint32_t bin_get(const uint8_t* p, const trailer_info* t, uint32_t i) {  /* reader.rs:30-48 */
    const uint8_t* q = p + t->bin_off + (size_t)i * t->step;
    return t->step == 2 ? get16(q) : get32(q);
}

/* parse_full / parse_truncated (data_block/mod.rs:58-191).  Returns 1 on an
 * item, 0 on the trailer marker, -status on error. */
static int parse_data_item(const uint8_t* p, size_t end, size_t* pos, int is_restart,
                           size_t base_key_off, uint64_t* seqno, uint32_t* key_off, uint16_t* key_len,
                           uint16_t* prefix_len, uint32_t* val_off, uint32_t* val_len, uint8_t* vt) {
    if (*pos > end) return -ORC_PARSE;
    uint8_t t = p[(*pos)++];
    if (t == TRAILER_MARKER) return (*pos - 1 == end) ? 0 : -ORC_PARSE;
    if (*pos > end || !valid_vtype(t)) return -ORC_PARSE;
    uint64_t v;
    if (rd_var(p, end, pos, 10, ~0ULL, &v)) return -ORC_PARSE;
    *seqno = v;
    uint64_t shared = 0, klen;
    if (!is_restart) {
        if (rd_var(p, end, pos, 3, 0xFFFF, &shared)) return -ORC_PARSE;
    }
    if (rd_var(p, end, pos, 3, 0xFFFF, &klen)) return -ORC_PARSE;
    if (*pos + klen > end) return -ORC_PARSE;
    if (!is_restart && base_key_off + shared > end) return -ORC_PARSE;
    *key_off = (uint32_t)*pos;
    *key_len = (uint16_t)klen;
    *prefix_len = (uint16_t)shared;
    *pos += klen;
    uint64_t vl = 0;
    if (!is_tombstone(t)) {
        if (rd_var(p, end, pos, 5, 0xFFFFFFFFULL, &vl)) return -ORC_PARSE;
    }
    if (*pos + vl > end) return -ORC_PARSE;
    *val_off = (uint32_t)*pos;
    *val_len = (uint32_t)vl;
    *pos += vl;
    *vt = t;
    return 1;
}

int64_t orc_data_block_decode(const uint8_t* p, size_t len, orc_parsed* out, uint64_t base,
                              uint64_t cap) {
    trailer_info t;
    if (read_trailer(p, len, &t)) return -ORC_PARSE;
    if (t.item_count > cap) return -ORC_OVERFLOW;
    size_t pos = 0, base_key_off = 0;
    uint32_t remaining = 0;          /* decoder.rs:54-58 LoScanner */
    uint64_t n = 0;
    for (;;) {
        int is_restart = remaining == 0;
        if (is_restart && n < t.item_count) {
            uint32_t r = (uint32_t)(n / t.ri);
            if (r >= t.bin_len || bin_get(p, &t, r) != pos) return -ORC_PARSE;
        }
        uint64_t seqno; uint32_t ko, vo, vl; uint16_t kl, pl; uint8_t vt;
        int rc = parse_data_item(p, t.rec_end, &pos, is_restart, base_key_off, &seqno, &ko, &kl, &pl,
                                 &vo, &vl, &vt);
        if (rc < 0) return rc;
        if (rc == 0) break;
        if (n >= t.item_count) return -ORC_PARSE;
        if (is_restart) base_key_off = ko;
        uint64_t k = base + n;
        if (out) {
            if (out->seqno) out->seqno[k] = seqno;
            if (out->key_off) out->key_off[k] = ko;
            if (out->val_off) out->val_off[k] = vo;
            if (out->val_len) out->val_len[k] = vl;
            if (out->key_len) out->key_len[k] = kl;
            if (out->prefix_len) out->prefix_len[k] = pl;
            if (out->vtype) out->vtype[k] = vt;
            if (out->handle_off) out->handle_off[k] = 0;
        }
        ++n;
        remaining = is_restart ? (uint32_t)t.ri - 1 : remaining - 1;
    }
    if (n != t.item_count) return -ORC_PARSE;
    return (int64_t)n;
}

int64_t orc_index_block_decode(const uint8_t* p, size_t len, orc_parsed* out, uint64_t base,
                               uint64_t cap) {
    trailer_info t;
    if (read_trailer(p, len, &t) || t.ri != 1) return -ORC_PARSE;
    if (t.item_count > cap) return -ORC_OVERFLOW;
    size_t pos = 0, end = t.rec_end;
    uint64_t n = 0;
    for (;;) {
        if (n < t.item_count && bin_get(p, &t, (uint32_t)n) != pos) return -ORC_PARSE;
        if (pos > end) return -ORC_PARSE;
        uint8_t m = p[pos++];
        if (m == TRAILER_MARKER) { if (pos - 1 != end) return -ORC_PARSE; break; }
        if (m != 0) return -ORC_PARSE;   /* block_handle.rs:140: marker is always 0 */
        uint64_t off, size, seqno, klen;
        if (rd_var(p, end, &pos, 10, ~0ULL, &off)) return -ORC_PARSE;
        if (rd_var(p, end, &pos, 5, 0xFFFFFFFFULL, &size)) return -ORC_PARSE;
        if (rd_var(p, end, &pos, 10, ~0ULL, &seqno)) return -ORC_PARSE;
        if (rd_var(p, end, &pos, 3, 0xFFFF, &klen)) return -ORC_PARSE;
        if (pos + klen > end) return -ORC_PARSE;
        if (n >= t.item_count) return -ORC_PARSE;
        uint64_t k = base + n;
        if (out) {
            if (out->seqno) out->seqno[k] = seqno;
            if (out->key_off) out->key_off[k] = (uint32_t)pos;
            if (out->val_off) out->val_off[k] = (uint32_t)(pos + klen);
            if (out->val_len) out->val_len[k] = (uint32_t)size;
            if (out->key_len) out->key_len[k] = (uint16_t)klen;
            if (out->prefix_len) out->prefix_len[k] = 0;
            if (out->vtype) out->vtype[k] = 0;
            if (out->handle_off) out->handle_off[k] = off;
        }
        pos += klen;
        ++n;
    }
    if (n != t.item_count) return -ORC_PARSE;
    return (int64_t)n;
}

/* compare_prefixed_slice (util.rs:133-167) */
static int cmp_bytes(const uint8_t* a, size_t an, const uint8_t* b, size_t bn) {
    size_t n = an < bn ? an : bn;
    int c = n ? memcmp(a, b, n) : 0;
    if (c) return c < 0 ? -1 : 1;
    return an < bn ? -1 : (an > bn ? 1 : 0);
}
static int cmp_prefixed(const uint8_t* pre, size_t pn, const uint8_t* suf, size_t sn,
                        const uint8_t* needle, size_t nn) {
    if (nn == 0) return (pn + sn) > 0 ? 1 : 0;
    size_t m = pn < nn ? pn : nn;
    int c = cmp_bytes(pre, m, needle, m);
    if (c) return c;
    if (pn > nn) return 1;
    return cmp_bytes(suf, sn, needle + m, nn - m);
}

int64_t orc_data_block_point_read(const uint8_t* p, size_t len, const uint8_t* needle,
                                  size_t nn, uint64_t snapshot) {
    trailer_info t;
    if (read_trailer(p, len, &t)) return -2;
    uint64_t n = t.item_count;
    orc_parsed o;
    uint64_t* sq = (uint64_t*)malloc(8 * (n ? n : 1));
    uint32_t* ko = (uint32_t*)malloc(4 * (n ? n : 1));
    uint16_t* kl = (uint16_t*)malloc(2 * (n ? n : 1));
    uint16_t* pl = (uint16_t*)malloc(2 * (n ? n : 1));
    memset(&o, 0, sizeof o);
    o.seqno = sq; o.key_off = ko; o.key_len = kl; o.prefix_len = pl;
    int64_t got = orc_data_block_decode(p, len, &o, 0, n);
    int64_t result = -1;
    if (got < 0) { result = -2; goto done; }
    /* Start item: hash probe (mod.rs:413-437) or restart binary search (iter.rs:37-76,
     * decoder.rs:153-207: last restart head with head_key < needle, else 0). */
    uint64_t start = 0;
    int use_search = 1;
    if (t.hash_len > 0) {
        /* the bucket bytes lie before the trailer (trailer.rs:100-111); a bucket naming a
         * restart interval the block does not have is malformed (the reference would index
         * past its binary index and panic) */
        if ((uint64_t)t.hash_off + t.hash_len > len - TRAILER_LEN) { result = -2; goto done; }
        uint32_t pos = (uint32_t)(orc_xxh3_64(needle, nn) % t.hash_len);
        uint8_t m = p[t.hash_off + pos];
        if (m == HASH_FREE) { result = -1; goto done; }
        if (m != HASH_CONFLICT) {
            if (m >= t.bin_len) { result = -2; goto done; }
            start = (uint64_t)m * t.ri;
            use_search = 0;
        }
    }
    if (use_search) {
        uint32_t lo = 0, hi = t.bin_len;
        while (lo < hi) {
            uint32_t mid = lo + (hi - lo) / 2;
            uint64_t h = (uint64_t)mid * t.ri;
            if (cmp_bytes(p + ko[h], kl[h], needle, nn) < 0) lo = mid + 1; else hi = mid;
        }
        uint32_t r = lo == 0 ? 0 : (lo == t.bin_len ? t.bin_len - 1 : lo - 1);
        start = (uint64_t)r * t.ri;
        /* Iter::seek linear scan stops at the first key >= needle (iter.rs:54-75);
         * the point_read loop below then continues from there. */
    }
    for (uint64_t i = start; i < n; ++i) {
        uint64_t h = (i / t.ri) * t.ri;
        int c = (i == h) ? cmp_bytes(p + ko[i], kl[i], needle, nn)
                         : cmp_prefixed(p + ko[h], pl[i], p + ko[i], kl[i], needle, nn);
        if (c > 0) break;
        if (c < 0) continue;
        if (sq[i] >= snapshot) continue;
        result = (int64_t)i;
        break;
    }
done:
    free(sq); free(ko); free(kl); free(pl);
    return result;
}

/* Iter::seek / seek_exclusive / seek_upper / seek_upper_exclusive
 * (data_block/iter.rs:37-176) over Decoder::partition_point (decoder.rs:153-207):
 * the restart interval is found by binary search over the restart heads, then a
 * linear scan (forward for the lower bound, backward from the interval's last
 * item for the upper bound) stops at the first key that ends the bound.  Result
 * = the item range [first, end) every iteration order yields, plus the two
 * return values.  Returns 0 or -status (malformed block). */
int orc_data_block_seek(const uint8_t* p, size_t len, const uint8_t* lo, size_t lo_len, const uint8_t* hi,
                        size_t hi_len, uint32_t flags, uint32_t* first, uint32_t* end, uint32_t* found) {
    trailer_info t;
    if (read_trailer(p, len, &t)) return -ORC_PARSE;
    uint64_t n = t.item_count;
    uint64_t* sq = (uint64_t*)malloc(8 * (n ? n : 1));
    uint32_t* ko = (uint32_t*)malloc(4 * (n ? n : 1));
    uint16_t* kl = (uint16_t*)malloc(2 * (n ? n : 1));
    uint16_t* pl = (uint16_t*)malloc(2 * (n ? n : 1));
    orc_parsed o;
    memset(&o, 0, sizeof o);
    o.seqno = sq; o.key_off = ko; o.key_len = kl; o.prefix_len = pl;
    int rc = 0;
    if (orc_data_block_decode(p, len, &o, 0, n) < 0) { rc = -ORC_PARSE; goto done; }
    uint64_t a = 0, b = n;
    uint32_t f = 0;
#define KEY_CMP(i, nd, nn) (((i) % t.ri == 0) ? cmp_bytes(p + ko[i], kl[i], nd, nn) \
        : cmp_prefixed(p + ko[((i) / t.ri) * t.ri], pl[i], p + ko[i], kl[i], nd, nn))
    if (flags & ORC_SEEK_LO) {
        /* partition_point(head < needle): last such head, else interval 0 */
        uint32_t l = 0, r = t.bin_len;
        while (l < r) {
            uint32_t mid = l + (r - l) / 2;
            uint64_t h = (uint64_t)mid * t.ri;
            if (cmp_bytes(p + ko[h], kl[h], lo, lo_len) < 0) l = mid + 1; else r = mid;
        }
        uint32_t iv = l == 0 ? 0 : (l == t.bin_len ? t.bin_len - 1 : l - 1);
        uint64_t i = (uint64_t)iv * t.ri;
        const int excl = (flags & ORC_SEEK_LO_EXCL) != 0;
        for (; i < n; ++i) {
            int c = KEY_CMP(i, lo, lo_len);
            if (!excl && c == 0) { f |= 1; break; }   /* Equal -> true */
            if (c > 0) { if (excl) f |= 1; break; }  /* Greater -> false (exclusive: true) */
        }
        a = i;
    }
    if (flags & ORC_SEEK_HI) {
        /* partition_point(head <= needle): last such head, else interval 0 */
        uint32_t l = 0, r = t.bin_len;
        while (l < r) {
            uint32_t mid = l + (r - l) / 2;
            uint64_t h = (uint64_t)mid * t.ri;
            if (cmp_bytes(p + ko[h], kl[h], hi, hi_len) <= 0) l = mid + 1; else r = mid;
        }
        uint32_t iv = l == 0 ? 0 : (l == t.bin_len ? t.bin_len - 1 : l - 1);
        uint64_t last = (uint64_t)(iv + 1) * t.ri;
        if (last > n) last = n;
        const int excl = (flags & ORC_SEEK_HI_EXCL) != 0;
        uint64_t e = last;  /* one past the item the backward scan stops at */
        for (; e > 0; --e) {
            int c = KEY_CMP(e - 1, hi, hi_len);
            if (!excl && c == 0) { f |= 2; break; }   /* Equal -> true */
            if (c < 0) { if (excl) f |= 2; break; }  /* Less -> false (exclusive: true) */
        }
        b = e;
    }
#undef KEY_CMP
    if (a > b) a = b;  /* the scanners crossed: an empty range */
    *first = (uint32_t)a;
    *end = (uint32_t)b;
    *found = f;
done:
    free(sq); free(ko); free(kl); free(pl);
    return rc;
}

uint64_t orc_cut_blocks(const orc_items* it, uint32_t block_size, uint32_t* starts,
                        uint64_t cap_blocks) {
    uint64_t nb = 0, chunk = 0, count = 0;
    if (it->n_items == 0) { if (cap_blocks) starts[0] = 0; return 0; }
    starts[0] = 0;
    for (uint64_t i = 0; i < it->n_items; ++i) {
        chunk += (it->key_off[i + 1] - it->key_off[i]) + (it->val_off[i + 1] - it->val_off[i]);
        ++count;
        if (chunk >= block_size) {       /* writer/mod.rs:284-290 */
            if (nb + 1 > cap_blocks) return nb;
            starts[++nb] = (uint32_t)(i + 1);
            chunk = 0;
            count = 0;
        }
    }
    if (count > 0) {                     /* finish() spills the rest, writer/mod.rs:374 */
        if (nb + 1 > cap_blocks) return nb;
        starts[++nb] = (uint32_t)it->n_items;
    }
    return nb;
}
