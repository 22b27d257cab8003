/*
 * lsm_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the fjall-rs/lsm-tree 3.1.9 SST block codec (the
 * `north_star` hot path).  It exists to CHECK the MI355X product path
 * (lsm-tree_amd/, include/lsmgpu.h) and to serve as the `cpu_baseline`
 * leg of bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline may load it.  The product never links or calls it.
 *
 * Every function names the reference file:line it restates.  The reference
 * is Rust and cannot be compiled in this image (no cargo/rustc), so parity is
 * pinned by the reference's own known-answer tests (src/hash.rs:17-31,
 * src/table/block/hash_index/mod.rs:49-79), the hand-derived block of
 * SURVEY.md Appendix B, and an independent Python restatement + python-xxhash
 * (libxxhash 0.8.2) — see tests/golden/make_golden.py.
 *
 * Third-party algorithms restated (absent from /root/reference):
 *   xxhash-rust ^0.8.15  (XXH3-64/128, seed 0, default 192-B secret)
 *   varint-rs   ^2.2.0   (unsigned LEB128)
 *   byteorder   (little-endian fixed width)
 */
#ifndef LSM_ORACLE_H
#define LSM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (mirror include/lsmgpu.h) ---------------------------- */
enum {
    ORC_OK = 0,
    ORC_BAD_MAGIC = 1,          /* Error::InvalidHeader("Block")  header.rs:125-127 */
    ORC_BAD_TYPE = 2,           /* Error::InvalidTag(("BlockType",v)) type.rs:33 */
    ORC_HDR_CKSUM = 3,          /* Error::ChecksumMismatch (header)   header.rs:156-161 */
    ORC_CKSUM = 4,              /* Error::ChecksumMismatch (payload)  block/mod.rs:94-102 */
    ORC_PARSE = 5,              /* reference panics (lib.rs:62-66); we report */
    ORC_OVERFLOW = 6,           /* caller buffer too small */
    ORC_TYPE_MISMATCH = 7,      /* block type != expected (util.rs:81-86) */
    ORC_TRUNCATED = 8,          /* handle shorter than header+data_length */
    ORC_UNSUPPORTED = 9,        /* compression != None */
    ORC_BAD_ARG = 10
};

/* ---- XXH3 (src/hash.rs:2-9 -> xxhash_rust::xxh3) ------------------------ */
uint64_t orc_xxh3_64(const uint8_t* p, size_t len);
void orc_xxh3_128(const uint8_t* p, size_t len, uint64_t* lo, uint64_t* hi);

/* ---- LEB128 (varint-rs) --------------------------------------------------- */
size_t orc_varint_len(uint64_t v);
size_t orc_varint_put(uint8_t* out, uint64_t v);

/* ---- items (SoA; identical layout to lsm_items in include/lsmgpu.h) ----- */
typedef struct orc_items {
    const uint8_t* keys;
    const uint64_t* key_off;  /* [n_items+1] */
    const uint8_t* vals;
    const uint64_t* val_off;  /* [n_items+1] */
    const uint64_t* seqno;    /* [n_items] */
    const uint8_t* vtype;     /* [n_items] */
    const uint64_t* handle_off;  /* index blocks: BlockHandle offset [n_items] */
    const uint32_t* handle_size; /* index blocks: BlockHandle size   [n_items] */
    uint64_t n_items;
} orc_items;

typedef struct orc_parsed {
    uint64_t* seqno;
    uint32_t* key_off;
    uint32_t* val_off;
    uint32_t* val_len;
    uint16_t* key_len;
    uint16_t* prefix_len;
    uint8_t* vtype;
    uint64_t* handle_off;
} orc_parsed;

/* DataBlock::encode_into (src/table/data_block/mod.rs:523-549) for items
 * [first, first+count).  Returns payload length or -status. */
int64_t orc_data_block_encode(const orc_items* it, uint64_t first, uint64_t count,
                              uint8_t restart_interval, float hash_ratio,
                              uint8_t* out, size_t cap);

/* IndexBlock::encode_into (src/table/index_block/mod.rs:110-127). */
int64_t orc_index_block_encode(const orc_items* it, uint64_t first, uint64_t count,
                               uint8_t* out, size_t cap);

/* Block::write_into, CompressionType::None (src/table/block/mod.rs:45-84).
 * Writes header(33)+payload; returns 33+len or -status. */
int64_t orc_block_write(const uint8_t* payload, size_t len, uint8_t block_type,
                        uint8_t* out, size_t cap);

typedef struct orc_header {
    uint8_t block_type;
    uint64_t cksum_lo, cksum_hi;
    uint32_t data_length;
    uint32_t uncompressed_length;
} orc_header;

/* Header::decode_from (src/table/block/header.rs:116-169). */
int orc_header_decode(const uint8_t* buf, size_t len, orc_header* h);

/* Block::from_file semantics over an in-memory handle (block/mod.rs:131-182):
 * header decode + xxh3_128 payload verify. */
int orc_block_verify(const uint8_t* buf, size_t len, orc_header* h);

/* Trailer item count (src/table/block/trailer.rs:57-75). */
int orc_trailer_item_count(const uint8_t* payload, size_t len, uint32_t* count);

/* Full forward Decoder::next iteration (src/table/block/decoder.rs:442-483)
 * of a data block payload: writes up to cap items at index base.. of `out`.
 * Returns the number of items parsed or -status. */
int64_t orc_data_block_decode(const uint8_t* payload, size_t len, orc_parsed* out,
                              uint64_t base, uint64_t cap);

/* Forward iteration of an index block (index_block/block_handle.rs:175-206). */
int64_t orc_index_block_decode(const uint8_t* payload, size_t len, orc_parsed* out,
                               uint64_t base, uint64_t cap);

/* DataBlock::point_read (src/table/data_block/mod.rs:412-472): returns the
 * item index in block order (0-based) or -1 if not found. */
int64_t orc_data_block_point_read(const uint8_t* payload, size_t len,
                                  const uint8_t* needle, size_t needle_len, uint64_t snapshot_seqno);

/* Iter::seek / seek_upper (+ _exclusive) (data_block/iter.rs:37-176): item range
 * [*first, *end) that iteration yields after the given bounds, *found bit 0 =
 * the lower seek's return value, bit 1 = the upper seek's.  0 or -status. */
#define ORC_SEEK_LO 1u
#define ORC_SEEK_HI 2u
#define ORC_SEEK_LO_EXCL 4u
#define ORC_SEEK_HI_EXCL 8u
int orc_data_block_seek(const uint8_t* payload, size_t len, const uint8_t* lo, size_t lo_len,
                        const uint8_t* hi, size_t hi_len, uint32_t flags, uint32_t* first,
                        uint32_t* end, uint32_t* found);

/* hash_index::Builder (hash_index/builder.rs:20-110): n set(key, idx) calls into
 * `buckets` bytes; Reader::get (hash_index/reader.rs:46-58). */
void orc_hash_index_build(const uint8_t* keys, const uint64_t* key_off, const uint8_t* idx, uint64_t n,
                          uint32_t buckets, uint8_t* out);
uint8_t orc_hash_index_get(const uint8_t* bytes, uint32_t buckets, const uint8_t* key, size_t klen);

/* Header::encode_into (header.rs:80-112) of arbitrary field values (33 bytes). */
void orc_header_encode(uint8_t block_type, uint64_t ck_lo, uint64_t ck_hi, uint32_t data_length,
                       uint32_t uncompressed_length, uint8_t* out);

/* Writer::write chunking (src/table/writer/mod.rs:243-296): block cut when
 * sum(key.len()+value.len()) >= block_size.  Writes n_blocks+1 starts;
 * returns n_blocks. */
uint64_t orc_cut_blocks(const orc_items* it, uint32_t block_size, uint32_t* block_item_start,
                        uint64_t cap_blocks);

/* Batched, multi-threaded CPU path (bench cpu_baseline + parity checker).
 * Encode: data blocks (block_type 0/3) or index blocks (1).  block_off gets
 * n_blocks+1 offsets into `out`.  Returns 0 or -status of first failure. */
int orc_encode_blocks(const orc_items* it, const uint32_t* block_item_start, uint32_t n_blocks,
                      uint8_t restart_interval, float hash_ratio, uint8_t block_type,
                      uint8_t* out, uint64_t cap, uint64_t* block_off, int nthreads);

/* Decode: verifies every block (header, checksums) and parses it.
 * item_start gets n_blocks+1 entries; status per block. */
int orc_decode_blocks(const uint8_t* blocks, const uint64_t* block_off, uint32_t n_blocks,
                      int expect_type, orc_parsed* out, uint64_t item_cap,
                      uint32_t* item_start, int32_t* status, int nthreads);

/* CPU-baseline "materialize" checksum: decode + rebuild every key
 * (Slice::fused(prefix, suffix), data_block/mod.rs:296-315) and fold a cheap
 * checksum so the work cannot be elided.  Returns items decoded. */
uint64_t orc_decode_materialize_blocks(const uint8_t* blocks, const uint64_t* block_off,
                                       uint32_t n_blocks, int nthreads, uint64_t* fold);

/* ---- standard Bloom filter (bloom.c; src/table/filter/standard_bloom/) ---- */
#define ORC_BLOOM_HDR 22 /* magic 4 + filter type 1 + hash type 1 + m u64 + k u64 */
uint64_t orc_bloom_calculate_m(uint64_t n, float fpr);
int orc_bloom_shape_fpr(uint64_t n, float fpr, uint64_t* m, uint64_t* k);
int orc_bloom_shape_bpk(uint64_t n, float bpk, uint64_t* m, uint64_t* k);
void orc_bloom_build(const uint64_t* hashes, uint64_t n, uint64_t m, uint64_t k, uint8_t* out);
int orc_bloom_contains(const uint8_t* filter, uint64_t len, uint64_t h1);

/* ---- LZ4 block format decoder (lz4.c; lz4_flex::decompress_into, block/mod.rs:104-118) ---- */
int64_t orc_lz4_decompress(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap);

#ifdef __cplusplus
}
#endif
#endif
