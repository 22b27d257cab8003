/*
 * lsmgpu.h — C ABI of the MI355X-native SST block codec (drop-in for the
 * fjall-rs/lsm-tree 3.1.9 block build/read API; see INTEGRATION.md for the
 * Rust `extern "C"` binding a maintainer would add).
 *
 * All entry points are batched: one call encodes or decodes many blocks in HBM.
 * Pointers named d_* are DEVICE pointers (hipMalloc'd, or torch CUDA tensors);
 * structs are passed by host pointer and hold device pointers.  `stream` is a
 * hipStream_t (NULL = default stream).  Every call is asynchronous on `stream`
 * and returns LSM_OK once the work is enqueued, or an argument error.
 * Per-block outcomes are written to d_status[] (lsm_status codes) on device.
 *
 * Reference interfaces replaced (paths relative to the reference repo):
 *   lsm_encode_blocks(32) <- DataBlock::encode_into src/table/data_block/mod.rs:523-549
 *                         IndexBlock::encode_into  src/table/index_block/mod.rs:110-127
 *                         Block::write_into        src/table/block/mod.rs:45-84
 *                         (per-block loop of Writer::spill_block, src/table/writer/mod.rs:303-337)
 *   lsm_decode_blocks  <- Block::from_file         src/table/block/mod.rs:131-182
 *                         Block::from_reader       src/table/block/mod.rs:87-128
 *                         load_block type check    src/table/util.rs:79-86
 *                         DataBlock::iter/Decoder  src/table/data_block/mod.rs:476, block/decoder.rs:442-483
 *                         IndexBlock::iter         src/table/index_block/mod.rs:91-95
 *   lsm_cut_blocks     <- Writer::write chunking   src/table/writer/mod.rs:243-296
 *   lsm_xxh3_128_batch <- hash128                  src/hash.rs:7-9 (checksum of arbitrary byte ranges)
 *   lsm_point_read_blocks <- DataBlock::point_read src/table/data_block/mod.rs:412-472
 *   lsm_seek_blocks    <- data_block::Iter::seek / seek_upper (+ _exclusive)  data_block/iter.rs:37-176
 *   lsm_xxh3_128_file  <- ChecksummedWriter         src/checksum.rs:59-96 (whole-file checksum)
 *   lsm_xxh3_128_stream_{init,update,digest}
 *                      <- ChecksummedWriter::{new,write,checksum} src/checksum.rs:59-96 (streaming)
 *   lsm_xxh3_128_stream_{init,update,digest}_batch
 *                      <- the same for every table of a MultiWriter  src/table/multi_writer.rs:181-257
 *   lsm_lz4_decompress_blocks <- Block::from_reader/from_file, CompressionType::Lz4  block/mod.rs:87-182
 *   lsm_lz4_plan_output <- the builder_unzeroed(uncompressed_length) sizing of the same  block/mod.rs:104-112
 *   lsm_lz4_plan_framed / lsm_lz4_decompress_framed + lsm_decode_blocks_tuned(LSM_DECODE_PAYLOAD_VERIFIED)
 *                      <- Block::from_reader(Lz4) then DataBlock::new + iter   block/mod.rs:104-118, data_block/mod.rs:335,476
 *   lsm_materialize_plan / lsm_materialize_keys <- DataBlockParsedItem::materialize  data_block/mod.rs:296-315
 *   lsm_scan_table     <- Scanner::new / next      src/table/scanner.rs:24-92 (block handles from the
 *                         block index: FullBlockIndex / TwoLevelBlockIndex, src/table/block_index/,
 *                         regions from the TOC, src/table/regions.rs:55-76)
 *   lsm_bloom_shape    <- BloomConstructionPolicy::init  src/table/filter/mod.rs:25-34
 *   lsm_hash64_keys    <- FullFilterWriter::register_key src/table/writer/filter/full.rs:47-50
 *   lsm_bloom_build    <- standard_bloom Builder set_with_hash + build  builder.rs:33-53,154-170
 *   lsm_bloom_contains <- StandardBloomFilterReader::contains_hash  standard_bloom/mod.rs:100-120
 */
#ifndef LSMGPU_H
#define LSMGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LSM_ABI_VERSION 7
#define LSM_HEADER_LEN 33  /* Header::serialized_len(), header.rs:64-76 */
#define LSM_TRAILER_LEN 31 /* TRAILER_SIZE, trailer.rs:14-23 */
/* d_blocks must be 16-byte aligned and readable for LSM_INPUT_PADDING bytes
 * past the last block (vector loads stage whole 16-byte granules). */
#define LSM_INPUT_PADDING 64

/* Per-block status.  Values mirror crate::Error (src/error.rs:134-167). */
typedef enum lsm_status {
    LSM_OK = 0,
    LSM_BAD_MAGIC = 1,     /* Error::InvalidHeader("Block")           header.rs:125-127 */
    LSM_BAD_TYPE = 2,      /* Error::InvalidTag(("BlockType", v))     type.rs:33 */
    LSM_HDR_CKSUM = 3,     /* Error::ChecksumMismatch (header)        header.rs:156-161 */
    LSM_CKSUM = 4,         /* Error::ChecksumMismatch (payload)       block/mod.rs:141-149 */
    LSM_PARSE = 5,         /* malformed payload: the reference panics (lib.rs:62-66) */
    LSM_OVERFLOW = 6,      /* output capacity exceeded */
    LSM_TYPE_MISMATCH = 7, /* Error::InvalidTag, block type != expected (util.rs:81-86) */
    LSM_TRUNCATED = 8,     /* handle shorter than header / data_length mismatch (Error::Io) */
    LSM_UNSUPPORTED = 9,   /* compression != None, filter block parse */
    LSM_BAD_ARG = 10,
    LSM_HIP_ERROR = 11,
    LSM_DECOMPRESS = 12,   /* Error::Decompress(Lz4): malformed LZ4 block   block/mod.rs:113-114 */
    /* Internal hand-off mark, never the result of a completed call: a streamed
     * huge-block checksum chain (lsm_decode_blocks_tuned, LSM_DECODE_HUGE_POOL,
     * blocks >= 2 MiB) stopped waiting for the parse units of its block (no
     * progress for 5 ms, e.g. other streams' kernels holding the CUs).  The
     * call's fallback chain pass recomputes every block so marked after the
     * parse kernel has ended and overwrites the mark with the block's real
     * status; only diagnostic builds can skip that pass.  It is not a
     * checksum mismatch (block/mod.rs:141-149 reports only real mismatches). */
    LSM_INCOMPLETE = 13
} lsm_status;

/* BlockType codes, src/table/block/type.rs:13-22 */
enum { LSM_BLOCK_DATA = 0, LSM_BLOCK_INDEX = 1, LSM_BLOCK_FILTER = 2, LSM_BLOCK_META = 3 };
/* ValueType codes, src/value_type.rs:36-58 */
enum { LSM_VALUE = 0, LSM_TOMBSTONE = 1, LSM_WEAK_TOMBSTONE = 2, LSM_INDIRECTION = 4 };

/* Encode input: the items of all blocks, in key order, as SoA arenas.
 * Item i: key = keys[key_off[i] .. key_off[i+1]), value likewise.
 * Data/meta blocks use keys, vals, seqno, vtype (InternalValue, value.rs:85-153).
 * Index blocks use keys (= end_key), seqno, handle_off, handle_size
 * (KeyedBlockHandle, index_block/block_handle.rs:67-80). */
typedef struct lsm_items {
    const uint8_t* keys;
    const uint64_t* key_off;     /* [n_items + 1] */
    const uint8_t* vals;
    const uint64_t* val_off;     /* [n_items + 1] */
    const uint64_t* seqno;       /* [n_items] */
    const uint8_t* vtype;        /* [n_items] ValueType code */
    const uint64_t* handle_off;  /* [n_items] index blocks only, else NULL */
    const uint32_t* handle_size; /* [n_items] index blocks only, else NULL */
    uint64_t n_items;
} lsm_items;

/* lsm_items with 32-bit key / value offsets (SURVEY 8(d)'s 4 + 4 bytes per item
 * instead of 8 + 8): for key and value arenas of less than 4 GiB each and fewer
 * than 2^32 - 1 items.  Same meaning, field for field; lsm_encode_blocks32. */
typedef struct lsm_items32 {
    const uint8_t* keys;
    const uint32_t* key_off;     /* [n_items + 1] */
    const uint8_t* vals;
    const uint32_t* val_off;     /* [n_items + 1] */
    const uint64_t* seqno;       /* [n_items] */
    const uint8_t* vtype;        /* [n_items] ValueType code */
    const uint64_t* handle_off;  /* [n_items] index blocks only, else NULL */
    const uint32_t* handle_size; /* [n_items] index blocks only, else NULL */
    uint64_t n_items;
} lsm_items32;

/* Decode output (mirrors DataBlockParsedItem / IndexBlockParsedItem,
 * data_block/mod.rs:272-316, index_block/mod.rs:24-62): payload-relative
 * SliceIndexes into each block's data (util.rs:26).  Item k of block b is
 * k in [item_start[b], item_start[b+1]).  NULL fields are not written.
 *   key     = payload[key_off .. key_off + key_len]  (suffix when truncated)
 *   prefix  = payload[head.key_off .. + prefix_len], head = first item of the
 *             restart interval (materialize: Slice::fused(prefix, key))
 *   value   = payload[val_off .. val_off + val_len]  (val_len 0 for tombstones)
 * Index blocks: vtype = 0, prefix_len = 0, val_len = BlockHandle size,
 *   handle_off = BlockHandle offset, val_off = end of the end_key. */
typedef struct lsm_parsed_items {
    uint64_t* seqno;
    uint32_t* key_off;
    uint32_t* val_off;
    uint32_t* val_len;
    uint16_t* key_len;
    uint16_t* prefix_len;
    uint8_t* vtype;
    uint64_t* handle_off;
} lsm_parsed_items;

/* Compact decode output (lsm_decode_blocks16): the same fields with 16-bit
 * payload offsets and lengths, 19 bytes per item instead of 25.  Only data and
 * meta blocks whose payload is at most 65535 bytes (every 4 / 16 KiB-target
 * block) are decoded into it; index blocks and larger payloads get
 * LSM_UNSUPPORTED (after the header and checksum checks, before the trailer). */
typedef struct lsm_parsed_items16 {
    uint64_t* seqno;
    uint16_t* key_off;
    uint16_t* val_off;
    uint16_t* val_len;
    uint16_t* key_len;
    uint16_t* prefix_len;
    uint8_t* vtype;
} lsm_parsed_items16;

typedef struct lsm_block_params {
    uint8_t restart_interval; /* data_block_restart_interval (config default 16); forced 1 for index */
    uint8_t block_type;       /* LSM_BLOCK_DATA / LSM_BLOCK_INDEX / LSM_BLOCK_META */
    uint8_t compression;      /* 0 = CompressionType::None (the only supported value) */
    uint8_t reserved;         /* must be 0 (else LSM_BAD_ARG) */
    float hash_ratio;         /* data_block_hash_ratio (default 0.0) */
    uint32_t flags;           /* LSM_ENCODE_HUGE_POOL | LSM_ENCODE_RUN_PLAN or 0; any other bit is LSM_BAD_ARG */
} lsm_block_params;
/* Take the workspace pool of lsm_encode_workspace_size_ex: blocks whose image
 * exceeds 96 KiB are written and hashed by work units across the whole GPU.
 * Without this flag the pool is never used, whatever the workspace size; with
 * it, a workspace too small for the pool's fixed part encodes without it. */
#define LSM_ENCODE_HUGE_POOL 1u
/* Plan each 32-block run inside the write kernel (block offsets by a decoupled
 * look-back across runs) instead of a plan pass and a size scan before it.  Taken
 * for data blocks without a hash index and without the pool, 1-512 items per
 * block on average; the library also takes it by itself at >= 128 items per block
 * (16 KiB blocks of short records: faster there, slower for 4 KiB blocks).  Same
 * bytes and statuses either way, except: a run whose predecessors' offsets do not
 * arrive within 100 ms (never seen) reports LSM_INCOMPLETE for its blocks and every
 * later run's, and an item_start array that is not strictly increasing rejects the
 * blocks of the 32-block run that holds the fault. */
#define LSM_ENCODE_RUN_PLAN 2u

/* Tuning knobs for the decode kernel (0 = library default).  Any flag bit
 * other than LSM_DECODE_ITEM_START_VALID / LSM_DECODE_PAYLOAD_VERIFIED /
 * LSM_DECODE_HUGE_POOL is rejected with LSM_BAD_ARG. */
typedef struct lsm_decode_tuning {
    uint32_t blocks_per_wave;  /* consecutive blocks one workgroup owns (1..63, default 54) */
    uint32_t stage_bytes;      /* LDS stage bytes (256..65536, default 34560); larger blocks take the general path */
    uint32_t tile_items;       /* items one stage may hold (default 480, at most 8192) */
    uint32_t flags;            /* LSM_DECODE_ITEM_START_VALID: d_item_start already holds the
                                  prefix sum of this batch (skip the count + scan pass) */
} lsm_decode_tuning;
#define LSM_DECODE_ITEM_START_VALID 1u
/* The payload checksums were verified upstream: skip the xxh3_128 of every
 * payload (header fields, data_length, type, trailer and records are still
 * checked).  For LZ4 blocks decompressed by lsm_lz4_decompress_framed, whose
 * stored bytes Block::from_reader verified before decompressing
 * (block/mod.rs:94-118); their frame headers carry the STORED checksum. */
#define LSM_DECODE_PAYLOAD_VERIFIED 2u
/* Take the workspace pool of lsm_decode_workspace_size_ex: blocks larger than
 * 72 KiB are cut into work units across the whole GPU.  Without this flag the
 * pool is never used, whatever the workspace size (lsm_decode_blocks, which
 * takes no tuning, never uses it); with it, the pool is used when the
 * workspace holds round_up(lsm_decode_workspace_size(n_blocks), 256) + 8704
 * bytes or more (smaller: decoded without it; a pool too small for every
 * huge block leaves the rest on the one-workgroup path). */
#define LSM_DECODE_HUGE_POOL 4u

/* Point-read results (DataBlock::point_read -> Option<InternalValue>,
 * data_block/mod.rs:412-472), one row per query; NULL fields other than item
 * are not written.  item = index of the hit in its block's item order (the
 * row lsm_decode_blocks gives it), -1 = None.  For a hit the key equals the
 * needle; the value is payload[val_off .. val_off + val_len). */
typedef struct lsm_point_result {
    int32_t* item;
    uint64_t* seqno;
    uint32_t* val_off;
    uint32_t* val_len;
    uint8_t* vtype;
} lsm_point_result;

int lsm_abi_version(void);
const char* lsm_status_name(int status);
/* Last HIP error string of this thread (after LSM_HIP_ERROR). */
const char* lsm_last_error(void);
int lsm_device_count(void);
int lsm_set_device(int device);

/* ---- decode ---------------------------------------------------------------
 * Verifies and parses n_blocks on-disk blocks (header || payload) located at
 * d_blocks[d_block_off[b] .. d_block_off[b+1]) (d_block_off: n_blocks+1
 * device u64, the BlockHandle offsets/sizes).  expect_type: block type every
 * block must have (util.rs:81-86), or -1 for any.  Writes d_item_start
 * (n_blocks+1 u32: prefix sum of the trailers' item counts, clamped at
 * item_cap), the parsed items, and d_status[n_blocks].  The rows
 * [d_item_start[b], d_item_start[b+1]) of a block whose d_status is not LSM_OK
 * are unspecified (blocks larger than the LDS stage are parsed chunk by chunk
 * while their checksum is still being computed, so a block that then fails it
 * may have rows written): as in the reference, where Block::from_file returns
 * Err and no item is yielded, a caller uses no row of a failed block.
 * d_workspace: lsm_decode_workspace_size(n_blocks) bytes of device memory, or,
 * with LSM_DECODE_HUGE_POOL in tuning->flags, lsm_decode_workspace_size_ex(n_blocks,
 * blocks_bytes) bytes (blocks_bytes >= the bytes the batch spans): then blocks
 * larger than 72 KiB (the writer's up-to-4-MiB data blocks, writer/mod.rs:193-198;
 * full block indexes) are cut into work units across the whole GPU instead of one
 * workgroup each.  Same outputs and statuses either way.  The pool is taken only
 * when the flag asks for it, never from the workspace size alone. */
size_t lsm_decode_workspace_size(uint32_t n_blocks);
size_t lsm_decode_workspace_size_ex(uint32_t n_blocks, uint64_t blocks_bytes);
int lsm_decode_blocks(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                      int32_t expect_type, const lsm_parsed_items* d_out, uint64_t item_cap,
                      uint32_t* d_item_start, int32_t* d_status, void* d_workspace,
                      size_t workspace_bytes, void* stream);
int lsm_decode_blocks_tuned(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                            int32_t expect_type, const lsm_parsed_items* d_out, uint64_t item_cap,
                            uint32_t* d_item_start, int32_t* d_status, void* d_workspace,
                            size_t workspace_bytes, const lsm_decode_tuning* tuning, void* stream);
/* lsm_decode_blocks_tuned into the compact 19 B/item layout (lsm_parsed_items16;
 * tuning may be NULL).  Same statuses, plus LSM_UNSUPPORTED for index blocks
 * and payloads over 65535 bytes.  Replaces the same decoder.rs:442-483 /
 * data_block/mod.rs:272-316 walk as lsm_decode_blocks. */
int lsm_decode_blocks16(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                        int32_t expect_type, const lsm_parsed_items16* d_out, uint64_t item_cap,
                        uint32_t* d_item_start, int32_t* d_status, void* d_workspace, size_t workspace_bytes,
                        const lsm_decode_tuning* tuning, void* stream);

/* ---- encode ---------------------------------------------------------------
 * Encodes n_blocks blocks; block b holds items [d_block_item_start[b],
 * d_block_item_start[b+1]) (n_blocks+1 device u32; every block non-empty,
 * mod.rs:530).  A d_block_item_start that is not strictly increasing is a
 * caller error: it gets LSM_BAD_ARG for some or all blocks of the batch (the
 * blocks planned together with the offending ones; every block when the batch
 * is planned item-parallel, >= 4 Ki items per block on average), so a caller
 * treats any LSM_BAD_ARG block as failing the whole batch.  Output blocks (header || payload) are packed back to back
 * into d_out; d_block_off (n_blocks+1 device u64) receives their offsets.
 * d_out needs lsm_encode_bound(...) bytes (status LSM_OVERFLOW otherwise).
 * d_workspace: lsm_encode_workspace_size(n_items, n_blocks) bytes, or, with
 * LSM_ENCODE_HUGE_POOL in params->flags, lsm_encode_workspace_size_ex(n_items,
 * n_blocks, out_cap) bytes: then blocks whose image exceeds 96 KiB (the writer's
 * up-to-4-MiB data blocks, writer/mod.rs:193-198) are written and hashed by work
 * units across the whole GPU instead of one workgroup each.  Same bytes either
 * way. */
uint64_t lsm_encode_bound(uint64_t n_items, uint32_t n_blocks, uint64_t key_bytes, uint64_t val_bytes,
                          const lsm_block_params* params);
size_t lsm_encode_workspace_size(uint64_t n_items, uint32_t n_blocks);
size_t lsm_encode_workspace_size_ex(uint64_t n_items, uint32_t n_blocks, uint64_t out_cap);
int lsm_encode_blocks(const lsm_items* d_items, const uint32_t* d_block_item_start, uint32_t n_blocks,
                      const lsm_block_params* params, uint8_t* d_out, uint64_t out_cap,
                      uint64_t* d_block_off, int32_t* d_status, void* d_workspace,
                      size_t workspace_bytes, void* stream);
/* lsm_encode_blocks over lsm_items32 (u32 key / value offsets): the same
 * kernels, bytes, statuses and workspace sizes; the item SoA the plan and write
 * passes read shrinks from 25 to 17 bytes per item. */
int lsm_encode_blocks32(const lsm_items32* d_items, const uint32_t* d_block_item_start, uint32_t n_blocks,
                        const lsm_block_params* params, uint8_t* d_out, uint64_t out_cap,
                        uint64_t* d_block_off, int32_t* d_status, void* d_workspace,
                        size_t workspace_bytes, void* stream);

/* ---- host-side helpers (no device work) ------------------------------------
 * Writer chunking on HOST arrays: cut a block when the running
 * sum(key_len + value_len) >= block_size (writer/mod.rs:284-290), the last
 * partial chunk is flushed as its own block (writer/mod.rs:374).  key_off and
 * val_off are host [n_items+1] arrays.  Writes block_item_start
 * (cap_blocks+1 entries) and returns the number of blocks. */
uint64_t lsm_cut_blocks(const uint64_t* key_off, const uint64_t* val_off, uint64_t n_items,
                        uint32_t block_size, uint32_t* block_item_start, uint64_t cap_blocks);

/* ---- checksums --------------------------------------------------------------
 * xxh3_128 (hash128, src/hash.rs:7-9) of n byte ranges
 * d_data[d_off[i] .. d_off[i+1]) into d_out (2 u64 per range: low, high). */
int lsm_xxh3_128_batch(const uint8_t* d_data, const uint64_t* d_off, uint32_t n, uint64_t* d_out,
                       void* stream);
/* Whole-file checksum: xxh3_128 of d_data[0 .. len) into d_out[0] (low), d_out[1]
 * (high), spread over the whole GPU (per-KiB contributions in parallel, then
 * the scramble chains: 8 waves, one accumulator each).  Replaces
 * ChecksummedWriter's streaming digest over an SST file held whole in HBM
 * (src/checksum.rs:59-96; equal to the one-shot xxh3_128,
 * tests/table_full_file_checksum.rs:26-31).  d_data readable up to 16 bytes
 * past len; workspace (16-byte aligned, any len incl. 0):
 * lsm_xxh3_128_file_workspace_size(len) bytes. */
size_t lsm_xxh3_128_file_workspace_size(uint64_t len);
int lsm_xxh3_128_file(const uint8_t* d_data, uint64_t len, uint64_t* d_out, void* d_workspace,
                      size_t workspace_bytes, void* stream);
/* The same checksum as a resumable stream, for a writer that emits the file
 * piece by piece (ChecksummedWriter::write per flushed region: data blocks,
 * then index, filter, meta and TOC, src/table/writer/mod.rs:66,99-102):
 *   init    ChecksummedWriter::new: a fresh running state in d_state
 *           (device memory, 16-byte aligned, lsm_xxh3_128_stream_state_size()
 *           bytes, caller-owned);
 *   update  ChecksummedWriter::write (checksum.rs:92-95): feed d_data[0 .. len)
 *           (device, any alignment, readable 16 bytes past len); workspace
 *           lsm_xxh3_128_stream_workspace_size(len) bytes, free again when
 *           the call's work on `stream` has finished;
 *   digest  ChecksummedWriter::checksum (Xxh3Default::digest128): xxh3_128 of
 *           everything fed so far into d_out[0..2] (low, high); the state is
 *           not changed, so updates may continue.
 * Any split of the input into updates gives the one-shot xxh3_128 of the
 * concatenation.  All three are asynchronous on `stream`; calls on one state
 * must be ordered (same stream, or events). */
size_t lsm_xxh3_128_stream_state_size(void);
size_t lsm_xxh3_128_stream_workspace_size(uint64_t len);
int lsm_xxh3_128_stream_init(void* d_state, void* stream);
int lsm_xxh3_128_stream_update(void* d_state, const uint8_t* d_data, uint64_t len, void* d_workspace,
                               size_t workspace_bytes, void* stream);
int lsm_xxh3_128_stream_digest(const void* d_state, uint64_t* d_out, void* stream);
/* The same for n running states at once (a flush or compaction that rotates
 * through several tables, src/table/multi_writer.rs:181-257, each with its own
 * ChecksummedWriter): d_states holds n states back to back (n *
 * lsm_xxh3_128_stream_state_size() bytes, 16-byte aligned, caller-owned).
 *   init_batch    ChecksummedWriter::new for every state;
 *   update_batch  state i is fed d_data[d_off[i] .. d_off[i+1]) (d_off: n+1
 *                 device u64, non-decreasing; empty ranges allowed; every
 *                 state at most once per call; the arena readable 16 bytes
 *                 past each range) in one launch sequence: the per-KiB
 *                 contributions of every state across the GPU, then 8 scramble
 *                 chains per state side by side.  total_len >= d_off[n] - d_off[0]
 *                 sizes the workspace (lsm_xxh3_128_stream_batch_workspace_size(n,
 *                 total_len) bytes, 16-byte aligned).  d_status[i] (device i32):
 *                 LSM_OK, or LSM_BAD_ARG for a state that was never initialised or
 *                 a decreasing range (that state is left unchanged); if the ranges
 *                 hold more bytes than total_len every state is LSM_BAD_ARG and
 *                 none is changed;
 *   digest_batch  d_out[2i], d_out[2i+1] = digest of state i (low, high). */
int lsm_xxh3_128_stream_init_batch(void* d_states, uint32_t n, void* stream);
size_t lsm_xxh3_128_stream_batch_workspace_size(uint32_t n, uint64_t total_len);
int lsm_xxh3_128_stream_update_batch(void* d_states, uint32_t n, const uint8_t* d_data, const uint64_t* d_off,
                                     uint64_t total_len, int32_t* d_status, void* d_workspace,
                                     size_t workspace_bytes, void* stream);
int lsm_xxh3_128_stream_digest_batch(const void* d_states, uint32_t n, uint64_t* d_out, void* stream);

/* ---- point read -----------------------------------------------------------
 * Batched DataBlock::point_read(needle, snapshot_seqno) (data_block/mod.rs:412-472),
 * the per-block step of Table::point_read (src/table/mod.rs:325-327): query q
 * looks up needle q (d_needles[d_needle_off[q] .. d_needle_off[q+1]), arena
 * readable LSM_INPUT_PADDING bytes past its end) in block d_query_block[q] of
 * the batch (same layout as lsm_decode_blocks; blocks of type Data or Meta, as
 * loaded and checksum-verified by Block::from_file).  Hash-index probe, else
 * restart binary search, then the MVCC linear scan (newest version with
 * seqno < snapshot).  d_status[q]: LSM_OK (hit or miss), or the structural
 * error of the block (LSM_PARSE, LSM_TRUNCATED, LSM_TYPE_MISMATCH, ...). */
int lsm_point_read_blocks(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                          const uint32_t* d_query_block, const uint8_t* d_needles,
                          const uint64_t* d_needle_off, const uint64_t* d_snapshot, uint32_t n_queries,
                          const lsm_point_result* d_out, int32_t* d_status, void* stream);

/* ---- range seek ------------------------------------------------------------
 * Batched data-block iterator bounds: Iter::seek / seek_exclusive (lower bound)
 * and Iter::seek_upper / seek_upper_exclusive (upper bound),
 * src/table/data_block/iter.rs:37-176 over Decoder::partition_point
 * (block/decoder.rs:153-207), the per-block step of Table::range
 * (src/table/mod.rs:391-422).  Query q seeks block d_query_block[q] (same
 * buffer rules as lsm_point_read_blocks) with the lower bound
 * d_lo[d_lo_off[q] .. d_lo_off[q+1]) and the upper bound
 * d_hi[d_hi_off[q] .. d_hi_off[q+1]) (arenas 16-byte aligned, readable
 * LSM_INPUT_PADDING bytes past their end), d_flags[q] saying which apply.
 * Result: items [d_first[q], d_end[q]) in block order (the rows
 * lsm_decode_blocks gives them) are exactly what next(), next_back() or any
 * mix of them yields; d_found[q] bit 0 / bit 1 = the return value of the lower
 * / upper seek (needle present, or for the exclusive forms: an item beyond
 * it).  d_status[q] as for lsm_point_read_blocks. */
#define LSM_SEEK_LO 1u            /* apply the lower bound */
#define LSM_SEEK_HI 2u            /* apply the upper bound */
#define LSM_SEEK_LO_EXCLUSIVE 4u  /* seek_exclusive: skip keys equal to the lower bound */
#define LSM_SEEK_HI_EXCLUSIVE 8u  /* seek_upper_exclusive: skip keys equal to the upper bound */
int lsm_seek_blocks(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                    const uint32_t* d_query_block, const uint8_t* d_lo, const uint64_t* d_lo_off,
                    const uint8_t* d_hi, const uint64_t* d_hi_off, const uint8_t* d_flags, uint32_t n_queries,
                    uint32_t* d_first, uint32_t* d_end, uint8_t* d_found, int32_t* d_status, void* stream);

/* ---- standard Bloom filter (src/table/filter/standard_bloom/) ---------------
 * The filter is the exact byte image of Builder::build (builder.rs:33-53):
 * "LSM\x03", filter type 0 (StandardBloom), hash type 0, m u64 LE, k u64 LE,
 * then m/8 bit bytes (bit i = byte i/8, mask 0x80 >> i%8,
 * bit_array/builder.rs:8-11).  Double hashing: h2 = (h1 >> 32) * 0x517cc1b727220a95,
 * position i = h1 % m, h1 += h2, h2 *= i for i = 1..k (builder.rs:10-13,154-170). */
enum { LSM_BLOOM_BITS_PER_KEY = 0, LSM_BLOOM_FP_RATE = 1 }; /* BloomConstructionPolicy */
#define LSM_BLOOM_HEADER 22
#define LSM_BLOOM_MAX_K 65536         /* larger k is rejected (bounded device loops) */
#define LSM_BLOOM_BAD_FILTER 0xFF     /* lsm_bloom_contains output: InvalidHeader("BloomFilter") */
/* Builder::calculate_m (builder.rs:128-151), f32 arithmetic as in the reference. */
uint64_t lsm_bloom_calculate_m(uint64_t n, float fpr);
/* (m, k) of BloomConstructionPolicy::{BitsPerKey(value), FalsePositiveRate(value)}.init(n)
 * (filter/mod.rs:25-34; with_bpk builder.rs:91-126, with_fp_rate :58-85).
 * LSM_BAD_ARG where the reference asserts (n == 0, bpk <= 0). */
int lsm_bloom_shape(uint64_t n, int policy, float value, uint64_t* m, uint64_t* k);
/* Byte length of the filter image: LSM_BLOOM_HEADER + m/8. */
uint64_t lsm_bloom_filter_size(uint64_t m);
/* hash64 = xxh3_64 (src/hash.rs:2-4) of n keys d_keys[d_key_off[i] .. d_key_off[i+1])
 * into d_out[i] (the FullFilterWriter hash buffer, writer/filter/full.rs:47-50).
 * d_keys 16-byte aligned and readable LSM_INPUT_PADDING bytes past its end. */
int lsm_hash64_keys(const uint8_t* d_keys, const uint64_t* d_key_off, uint64_t n, uint64_t* d_out, void* stream);
/* Builds the filter image of n hashes into d_filter (4-byte aligned, filter_cap >=
 * lsm_bloom_filter_size(m) rounded up to 4; the bytes past the image are zeroed).
 * m must be a positive multiple of 8 (both policies produce a multiple of 8; BitsPerKey < 1
 * gives m = 0, where the reference panics in h1 % m), 1 <= k <= LSM_BLOOM_MAX_K. */
int lsm_bloom_build(const uint64_t* d_hashes, uint64_t n, uint64_t m, uint64_t k, uint8_t* d_filter,
                    uint64_t filter_cap, void* stream);
/* d_out[i] = 1 if hash i may be contained, 0 if not (no false negatives),
 * LSM_BLOOM_BAD_FILTER if the image's header is malformed or truncated. */
int lsm_bloom_contains(const uint8_t* d_filter, uint64_t filter_len, const uint64_t* d_hashes, uint64_t n,
                       uint8_t* d_out, void* stream);

/* ---- LZ4 block decompression ----------------------------------------------
 * Block::from_reader / from_file with CompressionType::Lz4 (block/mod.rs:87-182),
 * batched: on-disk blocks d_blocks[d_block_off[b] .. d_block_off[b+1]) (header +
 * LZ4-compressed payload; same buffer rules as lsm_decode_blocks) are checked
 * (magic, type, header checksum, data_length, xxh3_128 of the stored payload) and
 * decompressed (lz4_flex::decompress_into, LZ4 block format) into
 * d_out[d_out_off[b] .. d_out_off[b+1]), whose length must be the header's
 * uncompressed_length (else LSM_OVERFLOW).  d_status[b]: LSM_OK, a header/checksum
 * status as in lsm_decode_blocks, or LSM_DECOMPRESS (malformed LZ4 stream, or one
 * that does not decode to exactly uncompressed_length bytes).
 * Workspace: lsm_lz4_workspace_size(n_blocks) bytes. */
size_t lsm_lz4_workspace_size(uint32_t n_blocks);
/* Output plan for lsm_lz4_decompress_blocks: d_out_off (n_blocks+1 device u64)
 * = exclusive prefix sum of each block's uncompressed_length, counted only for
 * blocks whose header verifies (magic, type, header checksum, data_length ==
 * handle size) and whose uncompressed_length <= max_block_bytes; other blocks
 * get 0 bytes (their decompress status is then the header error, or
 * LSM_OVERFLOW).  So a corrupt header cannot size the output, as
 * Block::from_reader allocates only after Header::decode_from passed
 * (block/mod.rs:91-112).  Workspace: lsm_lz4_plan_workspace_size(n_blocks). */
size_t lsm_lz4_plan_workspace_size(uint32_t n_blocks);
int lsm_lz4_plan_output(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                        uint64_t max_block_bytes, uint64_t* d_out_off, void* d_workspace, size_t workspace_bytes,
                        void* stream);
int lsm_lz4_decompress_blocks(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                              uint8_t* d_out, const uint64_t* d_out_off, int32_t* d_status,
                              void* d_workspace, size_t workspace_bytes, void* stream);

/* LZ4 -> parse chaining.  lsm_lz4_plan_framed is lsm_lz4_plan_output with 33
 * more bytes per verified block; lsm_lz4_decompress_framed writes each block
 * as a frame d_out[d_out_off[b] ..) = Header' || decompressed payload, where
 * Header' = the stored header with data_length = uncompressed_length and its
 * header checksum recomputed (the payload checksum field stays the STORED
 * bytes' checksum).  The frames are then decoded in place with
 * lsm_decode_blocks_tuned(d_out, d_out_off, ..., flags LSM_DECODE_PAYLOAD_VERIFIED);
 * a block's final status is its lsm_lz4_decompress_framed status if that is
 * not LSM_OK, else its decode status. */
int lsm_lz4_plan_framed(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                        uint64_t max_block_bytes, uint64_t* d_out_off, void* d_workspace, size_t workspace_bytes,
                        void* stream);
int lsm_lz4_decompress_framed(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                              uint8_t* d_out, const uint64_t* d_out_off, int32_t* d_status,
                              void* d_workspace, size_t workspace_bytes, void* stream);
/* lsm_lz4_plan_output (framed = 0) / lsm_lz4_plan_framed (framed = 1) for an output
 * arena the caller sized without reading the plan back (no host synchronisation):
 * when the planned bytes exceed out_cap every range is left empty, so the
 * decompress writes nothing and reports LSM_OVERFLOW for each block whose header
 * verifies (grow the arena and repeat). */
int lsm_lz4_plan_capped(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                        uint64_t max_block_bytes, int framed, uint64_t out_cap, uint64_t* d_out_off,
                        void* d_workspace, size_t workspace_bytes, void* stream);

/* ---- materialize (DataBlockParsedItem::materialize, data_block/mod.rs:296-315) --
 * Owned keys of decoded items: key = Slice::fused(prefix, suffix) =
 * payload[head.key_off .. + prefix_len] || payload[key_off .. + key_len], head =
 * the item's restart head (item - item % restart_interval within its block).
 * Values stay payload sub-slices (val_off, val_len), as in the reference.  Inputs
 * are lsm_decode_blocks' outputs (key_off, key_len, prefix_len required) over the
 * same blocks; n_items = d_item_start[n_blocks].  Items of blocks whose
 * d_status is not LSM_OK get empty keys.
 * lsm_materialize_plan: d_key_out_off (n_items+1 u64) = exclusive prefix sum of
 * the key lengths (workspace: lsm_materialize_workspace_size(n_items) bytes);
 * the caller sizes d_key_out from d_key_out_off[n_items], then
 * lsm_materialize_keys writes key i to d_key_out[d_key_out_off[i] .. [i+1]). */
size_t lsm_materialize_workspace_size(uint64_t n_items);
int lsm_materialize_plan(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                         const uint32_t* d_item_start, const int32_t* d_status, const lsm_parsed_items* d_parsed,
                         uint64_t n_items, uint64_t* d_key_out_off, void* d_workspace, size_t workspace_bytes,
                         void* stream);
int lsm_materialize_keys(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                         const uint32_t* d_item_start, const int32_t* d_status, const lsm_parsed_items* d_parsed,
                         uint64_t n_items, const uint64_t* d_key_out_off, uint8_t* d_key_out, void* stream);
/* lsm_materialize_keys into an arena of key_cap bytes sized without reading
 * d_key_out_off[n_items] back (no host synchronisation): every key is written
 * when they fit, none otherwise; *d_result (device i32) = LSM_OK or
 * LSM_OVERFLOW.  n_items may be the parsed arrays' capacity (items past
 * d_item_start[n_blocks] have empty keys). */
int lsm_materialize_keys_capped(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                                const uint32_t* d_item_start, const int32_t* d_status,
                                const lsm_parsed_items* d_parsed, uint64_t n_items, const uint64_t* d_key_out_off,
                                uint8_t* d_key_out, uint64_t key_cap, int32_t* d_result, void* stream);

/* ---- whole-table scan (Scanner, src/table/scanner.rs:24-92) -----------------
 * Decodes every data block of one table file image d_file[0 .. file_len) (16-byte
 * aligned, LSM_INPUT_PADDING readable bytes past file_len), in file order, as the
 * compaction read side does.  The block handles come from the table's block
 * index on the device: the TLI block (an index block at table->tli_off, size
 * table->tli_size: the "tli" TOC section, regions.rs:55-76) lists the data
 * blocks (FullBlockIndex, writer/index/full.rs:55-69) or, with
 * table->two_level (the TOC has an "index" section), index partitions that list
 * them (TwoLevelBlockIndex, writer/index/partitioned.rs:54-125).  The data
 * blocks must be contiguous from file offset 0 (the layout Scanner reads back to
 * back) and end inside the file.  Every item's seqno gets table->global_seqno
 * added (scanner.rs:84, wrapping).
 * Outputs: d_block_off (cap_blocks+1 u64: the data blocks, as lsm_decode_blocks
 * takes them), parsed items / d_item_start / d_status as lsm_decode_blocks
 * (block type Data expected, fetch_next_block scanner.rs:54-72),
 * *n_blocks (host) = number of data blocks, *table_status (host) = LSM_OK, or the
 * status of the first failing index block, LSM_OVERFLOW (more than cap_blocks
 * blocks or index entries), LSM_TRUNCATED (handles not contiguous from 0 or past
 * file_len) or LSM_PARSE (block count != table->block_count when non-zero,
 * the metadata's data_block_count).
 * Synchronises `stream` once per index level (the block count sizes the data
 * decode); the data decode itself is left enqueued on `stream`.
 * Workspace: lsm_scan_workspace_size(cap_blocks) bytes. */
typedef struct lsm_table_scan {
    uint64_t tli_off;       /* TLI region handle (TOC "tli" section) */
    uint32_t tli_size;
    uint32_t two_level;     /* 1: TLI entries are index partitions (TOC "index" section present) */
    uint64_t global_seqno;  /* Table::global_seqno, added to every item's seqno */
    uint64_t block_count;   /* ParsedMeta data_block_count (0 = not checked) */
} lsm_table_scan;
size_t lsm_scan_workspace_size(uint32_t cap_blocks);
int lsm_scan_table(const uint8_t* d_file, uint64_t file_len, const lsm_table_scan* table,
                   uint64_t* d_block_off, uint32_t cap_blocks, const lsm_parsed_items* d_out, uint64_t item_cap,
                   uint32_t* d_item_start, int32_t* d_status, uint32_t* n_blocks, int32_t* table_status,
                   void* d_workspace, size_t workspace_bytes, void* stream);
/* lsm_scan_table without host synchronisation: the entry counts stay on the
 * device and every level is launched for the caller's bounds (index_blocks_hint
 * index partitions of a two-level index, e.g. the TLI size / 4, else
 * cap_blocks; data_blocks_hint data blocks, e.g. the metadata's
 * data_block_count, else cap_blocks: keep them tight, the ranges past the real
 * counts are decoded as empty blocks; a level with more entries than its bound
 * gets LSM_OVERFLOW).  *d_n_blocks / *d_table_status (device)
 * receive what lsm_scan_table returns in *n_blocks / *table_status; a table
 * with more data blocks than the hint gets LSM_OVERFLOW.  d_item_start /
 * d_status hold data_blocks_hint (or cap_blocks) + 1 / entries: those past
 * *d_n_blocks are not meaningful.  Same workspace as lsm_scan_table. */
int lsm_scan_table_async(const uint8_t* d_file, uint64_t file_len, const lsm_table_scan* table,
                         uint64_t* d_block_off, uint32_t cap_blocks, uint32_t index_blocks_hint,
                         uint32_t data_blocks_hint, const lsm_parsed_items* d_out, uint64_t item_cap, uint32_t* d_item_start, int32_t* d_status,
                         uint32_t* d_n_blocks, int32_t* d_table_status, void* d_workspace, size_t workspace_bytes,
                         void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LSMGPU_H */
