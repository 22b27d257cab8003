// encode.hip — batched SST block encode on gfx950.
//
// Replaces, per block, DataBlock::encode_into / IndexBlock::encode_into
// (src/table/data_block/mod.rs:523-549, src/table/index_block/mod.rs:110-127,
// Encoder src/table/block/encoder.rs:84-164, Trailer trailer.rs:78-173) and
// Block::write_into (src/table/block/mod.rs:45-84, CompressionType::None):
// the payload xxh3_128 and the 33-byte header are fused into the same pass.
//
// Pipeline (all on one stream, DESIGN.md "Encode kernels"):
//   E1  size pass, one wave per block: per item (lane) the shared prefix
//       with the restart head (encoder.rs:140-143) and the record length;
//       wave scan -> records bytes, binary-index step, hash-index size.
//   S   device exclusive scan of block sizes -> d_block_off (packed output).
//   E2  write pass, one wave per block: key/value spans staged HBM->LDS in
//       coalesced 16 B/lane sweeps, each lane assembles its record in the LDS
//       payload image (dword stores inside records, byte stores at seams),
//       binary index, hash index (LDS min/max atomics reproduce the
//       order-independent FREE/idx/CONFLICT rule, hash_index/builder.rs:64-110),
//       trailer, wave xxh3_128 over the image, header, then one coalesced
//       16 B/lane copy-out to the block's place in the packed output.
//   E3  same algorithm straight on HBM for blocks whose staging does not fit
//       the LDS budget (grid-stride over a device list).
#include <hip/hip_runtime.h>

#include <math.h>

#include "block_format.hpp"
#include "decode.hpp"
#include "encode.hpp"
#include "scan.hpp"

namespace lsmgpu {

// Block classes by the LDS image a block needs (e2_need): small blocks are
// written by 4-wave workgroups with kImgSmall bytes of LDS per wave (8
// workgroups per CU), medium and big ones by listed 1-wave workgroups, and
// the rest straight in HBM (E3).
constexpr uint32_t kPlanHuge = 1, kPlanBad = 2, kPlanMedium = 4, kPlanBig = 8;
constexpr uint32_t kImgSmall = 5 * 1024;
constexpr uint32_t kImgMedium = 20 * 1024;
constexpr uint32_t kImgBig = 96 * 1024;
constexpr uint32_t kSmallWaves = 4;
constexpr uint32_t kE3HashChunk = 4096;    // buckets per LDS pass in E3
constexpr uint64_t kListedOne = 1ULL << 40, kOffMask = kListedOne - 1;

struct alignas(16) BlockPlan {
  uint32_t recs;      // bytes of all records
  uint32_t bin_len;   // restart heads
  uint32_t hash_w;    // buckets written (0 = no hash index in the block)
  uint32_t step_flags;  // step (2|4) | flags << 8
};

__device__ __forceinline__ uint32_t leb_len(uint64_t v) {
  const uint32_t bits = 64 - __builtin_clzll(v | 1);
  return (bits + 6) / 7;
}

// hash_index/builder.rs:39-63: (item_count as f32 * ratio) as u32, at least 1
__device__ __host__ __forceinline__ uint32_t bucket_count(uint64_t n, float ratio) {
  if (!(ratio > 0.0f)) return 0;
  const float prod = (float)n * ratio;
  uint32_t b;
  if (!(prod > 0.0f)) b = 0;
  else if (prod >= 4294967296.0f) b = 0xFFFFFFFFu;
  else b = (uint32_t)prod;
  return b < 1 ? 1 : b;
}

__device__ __forceinline__ Win16 read_win16_at(const uint8_t* base, uint64_t off) {
  return read_win16(base + (off & ~3ULL), (uint32_t)(off & 3));
}

// longest_shared_prefix_length, src/table/util.rs:125-130.  Up to 48 bytes
// per step with all six windows in flight together (one HBM round trip for
// the keys of every BASELINE shape).
__device__ __forceinline__ uint32_t lcp_global(const uint8_t* keys, uint64_t a, uint64_t b, uint32_t n) {
  uint32_t k = 0;
  while (k < n) {
    Win16 wa[3], wb[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      wa[i] = wb[i] = Win16{0, 0};
      if (i == 0 || k + 16 * i < n) {
        wa[i] = read_win16_at(keys, a + k + 16 * i);
        wb[i] = read_win16_at(keys, b + k + 16 * i);
      }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const uint32_t kk = k + 16 * i;
      if (kk >= n) return n;
      const uint64_t x0 = wa[i].lo ^ wb[i].lo, x1 = wa[i].hi ^ wb[i].hi;
      if (x0) return min(n, kk + (uint32_t)(__builtin_ctzll(x0) >> 3));
      if (x1) return min(n, kk + 8 + (uint32_t)(__builtin_ctzll(x1) >> 3));
    }
    k += 48;
  }
  return n;
}

struct EncodeParams {
  lsm_items it;
  const uint32_t* starts;
  uint32_t n_blocks;
  uint32_t ri;
  float ratio;
  uint32_t type;
  uint32_t diag;  // lsm_block_params.reserved: diagnostic ablations (0 in normal use)
  uint8_t* out;
  uint64_t out_cap;
  uint64_t* block_off;
  int32_t* status;
  uint16_t* shared;     // [n_items]
  uint64_t* sizes;      // [n_blocks] block bytes (E1) -> exclusive scan -> block_off
  BlockPlan* plans;     // [n_blocks]
  uint32_t* lists;      // [n_blocks]: the listed blocks in block order (from the size scan)
  uint32_t* list_count; // [1]
};

__device__ __forceinline__ bool is_index(const EncodeParams& P) { return P.type == 1; }

// LDS a block's image needs in E2: worst-case 16-B pad + the block + 32 B of
// read slack for the window reads, then the hash-index vote arrays.
__device__ __forceinline__ uint64_t e2_need(uint64_t total, uint32_t hash_w) {
  return ((15 + total + 15) & ~15ULL) + 32 + 8ULL * ((hash_w + 3) & ~3u);
}

// ------------------------------------------------------- record assembly
// Byte sink over a 4-aligned base: dword stores for bytes wholly inside the
// caller's record, byte stores at the seams shared with neighbour records.
struct ByteWriter {
  uint8_t* dst;
  uint32_t pos;
  uint64_t acc;
  uint32_t nacc;
  __device__ __forceinline__ void init(uint8_t* d, uint32_t p) { dst = d; pos = p; acc = 0; nacc = 0; }
  __device__ __forceinline__ void drain() {
    while (nacc && (pos & 3)) {
      dst[pos++] = (uint8_t)acc;
      acc >>= 8;
      --nacc;
    }
    if (nacc >= 4) {
      *reinterpret_cast<uint32_t*>(dst + pos) = (uint32_t)acc;
      acc >>= 32;
      nacc -= 4;
      pos += 4;
    }
  }
  __device__ __forceinline__ void byte(uint32_t b) {
    acc |= (uint64_t)(b & 0xFF) << (8 * nacc);
    ++nacc;
    if (nacc >= 4) drain();
  }
  __device__ __forceinline__ void word(uint32_t v, uint32_t n) {  // n in 1..4 low bytes of v
    if (n < 4) v &= (1u << (8 * n)) - 1;
    acc |= (uint64_t)v << (8 * nacc);
    nacc += n;
    if (nacc >= 4) drain();
  }
  __device__ __forceinline__ void leb(uint64_t v) {  // varint-rs write_*_varint
    while (v >= 0x80) {
      byte((uint32_t)(v & 0x7F) | 0x80);
      v >>= 7;
    }
    byte((uint32_t)v);
  }
  // n bytes from src_base[src_pos ..) (4-aligned base, any src_pos)
  __device__ __forceinline__ void copy(const uint8_t* src_base, uint32_t src_pos, uint32_t n) {
    uint32_t k = 0;
    for (; k + 4 <= n; k += 4) word(read_u32_unaligned(src_base, src_pos + k), 4);
    if (k < n) word(read_u32_unaligned(src_base, src_pos + k), n - k);
  }
  __device__ __forceinline__ void finish() {
    while (nacc) {
      dst[pos++] = (uint8_t)acc;
      acc >>= 8;
      --nacc;
    }
  }
};

// Span copy src (HBM, any alignment) -> dst[d .. d + n) (any alignment), in
// two steps so that all loads of a record are issued before its stores:
// load() reads the aligned 16-B windows that hold bytes of the span (the
// first K in registers; longer spans stream the rest at store time) and the
// at most 3 + 3 edge bytes; store() writes the destination dwords wholly
// inside the span (dword q, counted from d & ~3, is source bytes
// [base + 4q, base + 4q + 4) relative to the first window, base = (src & 15)
// - (d & 3), assembled with v_alignbyte) and the edge bytes, which share
// their dword with the neighbouring record.
template <int K>
struct SpanCopy {
  const u32x4* W;
  uint32_t n, d, rel, nwin, h, tl, hb, tb;
  u32x4 w[K];
  __device__ __forceinline__ void load(const uint8_t* src, uint32_t n_, uint32_t d_) {
    const uint64_t a = (uint64_t)(uintptr_t)src;
    W = reinterpret_cast<const u32x4*>(a & ~15ULL);
    n = n_;
    d = d_;
    rel = (uint32_t)(a & 15);
    nwin = n_ ? ((rel + n_ - 1) >> 4) + 1 : 0;
#pragma unroll
    for (int k = 0; k < K; ++k) w[k] = (uint32_t)k < nwin ? W[k] : u32x4{0, 0, 0, 0};
    h = min(n_, (4u - (d_ & 3u)) & 3u);
    tl = n_ > h ? (d_ + n_) & 3u : 0u;
    hb = tb = 0;
    for (uint32_t k = 0; k < h; ++k) hb |= (uint32_t)src[k] << (8 * k);
    for (uint32_t k = 0; k < tl; ++k) tb |= (uint32_t)src[n_ - tl + k] << (8 * k);
  }
  __device__ __forceinline__ void emit(uint8_t* dst, int wi, const u32x4& cw, uint32_t next0, int t0, uint32_t sh,
                                       uint32_t da, int qa, int qb) const {
    const uint32_t c[5] = {cw.x, cw.y, cw.z, cw.w, next0};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = 4 * wi + j - t0;
      if (q >= qa && q <= qb) *reinterpret_cast<uint32_t*>(dst + da + 4 * q) = alignbyte(c[j + 1], c[j], sh);
    }
  }
  __device__ __forceinline__ void store(uint8_t* dst) const {
    for (uint32_t k = 0; k < h; ++k) dst[d + k] = (uint8_t)(hb >> (8 * k));
    for (uint32_t k = 0; k < tl; ++k) dst[d + n - tl + k] = (uint8_t)(tb >> (8 * k));
    const int qa = (d & 3) ? 1 : 0;
    const int qb = (int)((d + n) >> 2) - (int)(d >> 2) - 1;
    if (!n || qb < qa) return;
    const int base = (int)rel - (int)(d & 3);
    const int t0 = base >> 2;  // -1 when the destination phase runs ahead of the source
    const uint32_t sh = (uint32_t)base & 3u;
    const uint32_t da = d & ~3u;
    // (t0 = -1 only when d & 3 > rel, and then dword 0 is an edge dword)
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if ((uint32_t)k < nwin) {
        uint32_t nx = 0;
        if (k + 1 < K) nx = w[k + 1].x;
        else if ((uint32_t)(k + 1) < nwin) nx = W[k + 1].x;
        emit(dst, k, w[k], nx, t0, sh, da, qa, qb);
      }
    }
    for (uint32_t k = K; k < nwin; ++k) {  // spans longer than K windows
      const u32x4 cw = W[k];
      const uint32_t nx = k + 1 < nwin ? W[k + 1].x : 0;
      emit(dst, (int)k, cw, nx, t0, sh, da, qa, qb);
    }
  }
};

// One item's fields, loaded once per lane (all loads independent).
struct ItemMeta {
  uint64_t ko, vo, seq;
  uint32_t klen, vl, vt, sh;
};

__device__ __forceinline__ ItemMeta load_item(const EncodeParams& P, uint64_t i, bool& bad) {
  ItemMeta m;
  m.ko = P.it.key_off[i];
  const uint64_t kl = P.it.key_off[i + 1] - m.ko;
  if (kl > 0xFFFF) bad = true;
  m.klen = (uint32_t)min(kl, (uint64_t)0xFFFF);
  m.seq = P.it.seqno[i];
  m.sh = 0;
  if (is_index(P)) {
    m.vo = P.it.handle_off[i];
    m.vl = P.it.handle_size[i];
    m.vt = 0;
  } else {
    m.vo = P.it.val_off[i];
    const uint64_t vl = P.it.val_off[i + 1] - m.vo;
    m.vt = P.it.vtype[i];
    if (!valid_vtype(m.vt)) bad = true;
    if (!is_tombstone(m.vt) && vl > 0xFFFFFFFFULL) bad = true;
    m.vl = (uint32_t)vl;
  }
  return m;
}

// Item j of the block starting at item s, with its shared prefix against the
// restart head (encoder.rs:140-143, util.rs:125-130).
__device__ __forceinline__ ItemMeta load_item_lcp(const EncodeParams& P, uint32_t s, uint32_t j, uint32_t ri,
                                                  bool& bad) {
  const uint64_t i = (uint64_t)s + j;
  ItemMeta m = load_item(P, i, bad);
  if (!is_index(P) && j % ri != 0) {
    const uint64_t h = (uint64_t)s + (j / ri) * ri;
    const uint64_t hko = P.it.key_off[h];
    const uint32_t hkl = (uint32_t)min(P.it.key_off[h + 1] - hko, (uint64_t)0xFFFF);
    m.sh = lcp_global(P.it.keys, hko, m.ko, min(hkl, m.klen));
  }
  return m;
}

__device__ __forceinline__ uint32_t head_len(const EncodeParams& P, const ItemMeta& m, bool head) {
  if (is_index(P)) return 1 + leb_len(m.vo) + leb_len(m.vl) + leb_len(m.seq) + leb_len(m.klen);
  return 1 + leb_len(m.seq) + (head ? leb_len(m.klen) : leb_len(m.sh) + leb_len(m.klen - m.sh));
}

__device__ __forceinline__ uint64_t item_record_len(const EncodeParams& P, const ItemMeta& m, bool head) {
  uint64_t rec = head_len(P, m, head) + m.klen - (head ? 0 : m.sh);
  if (!is_index(P) && !is_tombstone(m.vt)) rec += leb_len(m.vl) + (uint64_t)m.vl;
  return rec;
}

// Byte stores of a LEB128 (varint-rs write_*_varint) / single bytes.
__device__ __forceinline__ uint32_t put_leb(uint8_t* dst, uint32_t pos, uint64_t v) {
  while (v >= 0x80) {
    dst[pos++] = (uint8_t)(v | 0x80);
    v >>= 7;
  }
  dst[pos++] = (uint8_t)v;
  return pos;
}

// One record at dpos: issue() loads the key (suffix) and value spans, store()
// writes the record (encode_full_into / encode_truncated_into,
// data_block/mod.rs:195-264; index: block_handle.rs:134-156).
struct RecordCopy {
  SpanCopy<2> key;
  SpanCopy<5> val;
  uint32_t dpos;
  __device__ __forceinline__ void issue(const EncodeParams& P, const ItemMeta& m, bool head, uint32_t dpos_) {
    dpos = dpos_;
    const uint32_t kfrom = head ? 0 : m.sh;
    const uint32_t kpos = dpos_ + head_len(P, m, head);
    key.load(P.it.keys + m.ko + kfrom, m.klen - kfrom, kpos);
    const bool has_val = !is_index(P) && !is_tombstone(m.vt);
    const uint32_t vpos = kpos + m.klen - kfrom + leb_len(m.vl);
    val.load(P.it.vals + (has_val ? m.vo : 0), has_val ? m.vl : 0, vpos);
  }
  __device__ __forceinline__ void store(const EncodeParams& P, const ItemMeta& m, bool head, uint8_t* dst) const {
    uint32_t pos = dpos;
    if (is_index(P)) {
      dst[pos++] = 0;
      pos = put_leb(dst, pos, m.vo);
      pos = put_leb(dst, pos, m.vl);
      pos = put_leb(dst, pos, m.seq);
      put_leb(dst, pos, m.klen);
    } else {
      dst[pos++] = (uint8_t)m.vt;
      pos = put_leb(dst, pos, m.seq);
      if (head) {
        put_leb(dst, pos, m.klen);
      } else {
        pos = put_leb(dst, pos, m.sh);
        put_leb(dst, pos, m.klen - m.sh);
      }
      if (!is_tombstone(m.vt)) put_leb(dst, key.d + key.n, m.vl);
    }
    key.store(dst);
    val.store(dst);
  }
};

__device__ __forceinline__ void store_le(uint8_t* dst, uint32_t pos, uint64_t v, uint32_t n) {
  for (uint32_t k = 0; k < n; ++k) dst[pos + k] = (uint8_t)(v >> (8 * k));
}

// Hash-index bucket of a key (hash_index/mod.rs:35-41), key bytes from HBM.
__device__ __forceinline__ uint32_t key_bucket(const EncodeParams& P, uint64_t ko, uint32_t klen, uint32_t buckets) {
  const uint64_t ka = (uint64_t)(uintptr_t)P.it.keys + ko;
  const uint8_t* kb = reinterpret_cast<const uint8_t*>(ka & ~15ULL);
  const uint32_t kq = (uint32_t)(ka & 15);
  const uint64_t h = xxh3_64_any(klen, BaseReader8{kb, kq}, BaseReader64{kb, kq});
  return (uint32_t)(h % buckets);
}

// Marker, binary index entries are written by the record loop; this writes
// the hash-index bytes (given final min/max per bucket) and the trailer.
__device__ __forceinline__ uint32_t bucket_byte(uint32_t lo, uint32_t hi) {
  return lo == 0xFFFFFFFFu ? kHashFree : (lo == hi ? lo : kHashConflict);
}

__device__ __forceinline__ void write_trailer_bytes(uint8_t* dst, uint32_t tp, uint32_t ri, uint32_t step,
                                                    uint32_t bin_len, uint32_t bin_off, uint32_t hash_w,
                                                    uint32_t hash_off, uint32_t items) {
  // trailer.rs:118-163, lanes 0..30 write one byte each
  const int lane = threadIdx.x & 63;
  if (lane >= (int)kTrailerLen) return;
  uint32_t v;
  const int k = lane;
  if (k == 0) v = ri;
  else if (k == 1) v = step;
  else if (k < 6) v = bin_len >> (8 * (k - 2));
  else if (k < 10) v = bin_off >> (8 * (k - 6));
  else if (k < 14) v = hash_w >> (8 * (k - 10));
  else if (k < 18) v = hash_off >> (8 * (k - 14));
  else if (k == 18) v = 1;       // prefix truncation on
  else if (k < 27) v = 0;        // fixed key/value size (unused)
  else v = items >> (8 * (k - 27));
  dst[tp + k] = (uint8_t)v;
}

// Header::encode_into (header.rs:80-112): lanes 0..32 write one byte each.
__device__ __forceinline__ void write_header_bytes(uint8_t* dst, uint32_t hp, uint32_t type, uint64_t ck_lo,
                                                   uint64_t ck_hi, uint32_t plen) {
  uint64_t w0 = 0x034D534CULL | ((uint64_t)type << 32) | (ck_lo << 40);
  uint64_t w1 = (ck_lo >> 24) | (ck_hi << 40);
  uint64_t w2 = (ck_hi >> 24) | ((uint64_t)plen << 40);
  uint64_t w3 = ((uint64_t)plen >> 24) | ((uint64_t)plen << 8);
  auto r64 = [&](uint32_t o) -> uint64_t {  // LE u64 at byte o of w0..w3 (o <= 24)
    const uint32_t q = o >> 3, sft = (o & 7) * 8;
    const uint64_t a = q == 0 ? w0 : q == 1 ? w1 : q == 2 ? w2 : w3;
    const uint64_t b = q == 0 ? w1 : q == 1 ? w2 : q == 2 ? w3 : 0;
    return sft ? (a >> sft) | (b << (64 - sft)) : a;
  };
  auto r8 = [&](uint32_t o) -> uint32_t { return (uint32_t)(r64(o) & 0xFF); };
  uint64_t hlo, hhi;
  xxh3_128_short(29, r8, r64, hlo, hhi);
  const int lane = threadIdx.x & 63;
  if (lane < 29) dst[hp + lane] = (uint8_t)r8(lane);
  else if (lane < 33) dst[hp + lane] = (uint8_t)((uint32_t)hlo >> (8 * (lane - 29)));
}

// ------------------------------------------------------ E2: LDS write pass
// Wave-local ordering of LDS traffic between lanes (no workgroup barrier:
// the waves of a workgroup write independent blocks).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

// Block tail in the image: marker, hash-index bytes, trailer, then the fused
// xxh3_128 + header, and one coalesced 16 B/lane copy-out to the block's
// place in the packed output.
__device__ __forceinline__ void finish_block_lds(const EncodeParams& P, uint32_t b, const BlockPlan& pl, uint32_t n,
                                                 uint32_t ri, uint8_t* img, const uint32_t* hlo, const uint32_t* hhi,
                                                 uint32_t pad, uint32_t total, uint8_t* gdst) {
  const int lane = threadIdx.x & 63;
  const uint32_t step = pl.step_flags & 0xFF;
  const uint32_t plen = total - kHdrLen, p0 = pad + kHdrLen, bin_off = pl.recs + 1;
  if (lane == 0) img[p0 + pl.recs] = kTrailerMarker;
  const uint32_t hash_off = pl.hash_w ? bin_off + pl.bin_len * step : 0;
  for (uint32_t k = lane; k < pl.hash_w; k += kWave) img[p0 + hash_off + k] = (uint8_t)bucket_byte(hlo[k], hhi[k]);
  write_trailer_bytes(img, p0 + plen - kTrailerLen, ri, step, pl.bin_len, bin_off, pl.hash_w, hash_off, n);
  wave_lds_sync();
  if (!(kDiagBuild && (P.diag & 2))) {
    uint64_t ck_lo, ck_hi;
    xxh3_128_wave(img, p0, plen, &kLongSecret, ck_lo, ck_hi);
    write_header_bytes(img, pad, P.type, ck_lo, ck_hi, plen);
  }
  wave_lds_sync();
  const uint32_t chunks = (kDiagBuild && (P.diag & 4)) ? 0 : (pad + total + 15) >> 4;
  for (uint32_t c = lane; c < chunks; c += kWave) {
    const uint32_t lo = c * 16, hi = lo + 16;
    if (lo >= pad && hi <= pad + total) {
      // streaming output: non-temporal (measured 2 % faster than a plain store)
      __builtin_nontemporal_store(reinterpret_cast<const u32x4*>(img)[c], reinterpret_cast<u32x4*>(gdst) + c);
    } else {
      for (uint32_t k = max(lo, pad); k < min(hi, pad + total); ++k) gdst[k] = img[k];
    }
  }
  if (lane == 0) P.status[b] = ST_OK;
}

// Listed block b (any item count) assembled by one wave in the LDS image at
// `smem` (16-B aligned, at least e2_need bytes); shared prefixes and the plan
// come from the fused pass.
__device__ __forceinline__ void write_block_lds(const EncodeParams& P, uint32_t b, uint8_t* smem) {
  const int lane = threadIdx.x & 63;
  const uint32_t s = P.starts[b], e = P.starts[b + 1];
  const uint64_t dst_off = P.block_off[b], dst_end = P.block_off[b + 1];
  const BlockPlan pl = P.plans[b];
  const uint32_t step = pl.step_flags & 0xFF;
  if (dst_end > P.out_cap) {
    if (lane == 0) P.status[b] = ST_OVERFLOW;
    return;
  }
  const uint32_t n = e - s;
  const uint32_t ri = is_index(P) ? 1 : P.ri;
  const uint32_t total = (uint32_t)(dst_end - dst_off);
  const uint64_t dabs = (uint64_t)(uintptr_t)P.out + dst_off;
  const uint32_t pad = (uint32_t)(dabs & 15);
  uint8_t* img = smem;
  uint32_t* hlo = reinterpret_cast<uint32_t*>(smem + ((pad + total + 15) & ~15u) + 32);
  uint32_t* hhi = hlo + ((pl.hash_w + 3) & ~3u);
  for (uint32_t k = lane; k < pl.hash_w; k += kWave) {
    hlo[k] = 0xFFFFFFFFu;
    hhi[k] = 0;
  }
  wave_lds_sync();
  const uint32_t p0 = pad + kHdrLen;
  const uint32_t bin_off = pl.recs + 1;
  uint32_t carry = 0;
  for (uint32_t c = 0; c < n; c += kWave) {
    const uint32_t j = c + lane;
    const uint64_t i = (uint64_t)s + j;
    const bool head = j % ri == 0;
    ItemMeta m;
    RecordCopy rc;
    uint32_t rec = 0;
    if (j < n) {
      bool bad = false;
      m = load_item(P, i, bad);
      if (!is_index(P)) m.sh = P.shared[i];
      rec = (uint32_t)item_record_len(P, m, head);
    }
    const uint32_t incl = wave_incl_scan_u32(rec);
    const uint32_t roff = carry + incl - rec;
    if (j < n) {
      rc.issue(P, m, head, p0 + roff);
      rc.store(P, m, head, img);
      if (head) store_le(img, p0 + bin_off + (j / ri) * step, roff, step);
      if (pl.hash_w) {
        const uint32_t bk = key_bucket(P, m.ko, m.klen, pl.hash_w);
        atomicMin(&hlo[bk], j / ri);
        atomicMax(&hhi[bk], j / ri);
      }
    }
    carry += wave_bcast_u32(incl, 63);
  }
  wave_lds_sync();
  finish_block_lds(P, b, pl, n, ri, img, hlo, hhi, pad, total, reinterpret_cast<uint8_t*>(dabs & ~15ULL));
}

// ---------------------------------------------------------------- E1: sizes
// One wave per block: item fields, shared prefixes (stored for E2) and record
// sizes -> block bytes, binary-index step, hash-index size, size class.
__global__ __launch_bounds__(256) void encode_sizes_kernel(EncodeParams P) {
  const int lane = threadIdx.x & 63;
  const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= P.n_blocks) return;
  const uint32_t s = P.starts[b], e = P.starts[b + 1];
  const uint32_t ri = is_index(P) ? 1 : P.ri;
  bool bad = e <= s;
  const uint32_t n = bad ? 0 : e - s;
  uint64_t carry = 0, last_head = 0;
  const uint32_t lh = n ? ((n - 1) / ri) * ri : 0;
  for (uint32_t c = 0; c < n; c += kWave) {
    const uint32_t j = c + lane;
    uint64_t rec = 0;
    if (j < n) {
      const ItemMeta m = load_item_lcp(P, s, j, ri, bad);
      if (!is_index(P)) P.shared[(uint64_t)s + j] = (uint16_t)m.sh;
      rec = item_record_len(P, m, j % ri == 0);
    }
    const uint64_t incl = wave_incl_scan_u64(rec);
    if (lh >= c && lh < c + kWave) last_head = carry + wave_bcast_u64(incl - rec, lh - c);
    carry += wave_bcast_u64(incl, 63);
  }
  bad = __ballot(bad) != 0;
  if (lane != 0) return;
  const uint32_t bin_len = n ? (n + ri - 1) / ri : 0;
  const uint32_t step = last_head <= 0xFFFF ? 2 : 4;
  const uint32_t buckets = is_index(P) ? 0 : bucket_count(n, P.ratio);
  const uint32_t hash_w = (buckets > 0 && bin_len <= kHashMaxPointers) ? buckets : 0;
  const uint64_t total = kHdrLen + carry + 1 + (uint64_t)bin_len * step + hash_w + kTrailerLen;
  if (carry > 0xFFFFFFF0ULL || total > 0xFFFFFF00ULL) bad = true;
  uint32_t flags = 0;
  if (bad) {
    flags = kPlanBad;
    P.status[b] = ST_BAD_ARG;
  } else {
    const uint64_t need = e2_need(total, hash_w);
    if (need > kImgSmall || n > kWave)
      flags = need <= kImgMedium ? kPlanMedium : need <= kImgBig ? kPlanBig : kPlanHuge;
  }
  P.plans[b] = BlockPlan{(uint32_t)carry, bin_len, hash_w, step | (flags << 8)};
  // bits 40.. count the listed (not small) blocks: the size scan numbers them
  // (no global atomics: one counter serialised a batch of uniformly large blocks)
  P.sizes[b] = (bad ? 0 : total) | ((flags & (kPlanMedium | kPlanBig | kPlanHuge)) ? kListedOne : 0);
}

// ------------------------------------------------- E2: small blocks in LDS
// kSmallWaves waves per workgroup, one block (<= 64 items, image <= kImgSmall)
// per wave, lane = item: all of a lane's loads (item fields, key and value
// windows) are in flight together, then the record is stored into the image.
#ifndef LSM_ENC_WPE
#define LSM_ENC_WPE 5
#endif
__global__ __launch_bounds__(kSmallWaves * kWave) __attribute__((amdgpu_waves_per_eu(LSM_ENC_WPE))) void encode_write_kernel(EncodeParams P) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const uint32_t b = blockIdx.x * kSmallWaves + wave;
  if (b >= P.n_blocks) return;
  const BlockPlan pl = P.plans[b];
  if ((pl.step_flags >> 8) != 0) return;  // listed (medium / big / huge) or rejected
  const uint32_t s = P.starts[b], n = P.starts[b + 1] - s;
  const uint64_t off = P.block_off[b], end = P.block_off[b + 1];
  if (end > P.out_cap) {
    if (lane == 0) P.status[b] = ST_OVERFLOW;
    return;
  }
  const uint32_t ri = is_index(P) ? 1 : P.ri;
  const uint32_t step = pl.step_flags & 0xFF;
  const uint32_t total = (uint32_t)(end - off);
  const uint64_t dabs = (uint64_t)(uintptr_t)P.out + off;
  const uint32_t pad = (uint32_t)(dabs & 15);
  const uint32_t p0 = pad + kHdrLen;
  const bool head = lane % ri == 0;
  ItemMeta m;
  RecordCopy rc;
  uint32_t rec = 0;
  if ((uint32_t)lane < n) {
    bool bad = false;
    m = load_item(P, (uint64_t)s + lane, bad);
    if (!is_index(P)) m.sh = P.shared[(uint64_t)s + lane];
    rec = (uint32_t)item_record_len(P, m, head);
  }
  const uint32_t roff = wave_incl_scan_u32(rec) - rec;
  if ((uint32_t)lane < n) rc.issue(P, m, head, p0 + roff);
  uint8_t* img = smem + wave * kImgSmall;
  uint32_t* hlo = reinterpret_cast<uint32_t*>(img + ((pad + total + 15) & ~15u) + 32);
  uint32_t* hhi = hlo + ((pl.hash_w + 3) & ~3u);
  for (uint32_t k = lane; k < pl.hash_w; k += kWave) {
    hlo[k] = 0xFFFFFFFFu;
    hhi[k] = 0;
  }
  wave_lds_sync();
  if ((uint32_t)lane < n && !(kDiagBuild && (P.diag & 1))) {
    rc.store(P, m, head, img);
    if (head) store_le(img, p0 + pl.recs + 1 + (lane / ri) * step, roff, step);
    if (pl.hash_w) {
      const uint32_t bk = key_bucket(P, m.ko, m.klen, pl.hash_w);
      atomicMin(&hlo[bk], lane / ri);
      atomicMax(&hhi[bk], lane / ri);
    }
  }
  wave_lds_sync();
  finish_block_lds(P, b, pl, n, ri, img, hlo, hhi, pad, total, reinterpret_cast<uint8_t*>(dabs & ~15ULL));
}

// Listed medium / big blocks: one wave per workgroup, grid-stride over the list.
__global__ __launch_bounds__(kWave) void encode_write_list_kernel(EncodeParams P, uint32_t plan_flag) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t count = P.list_count[0];
  for (uint32_t li = blockIdx.x; li < count; li += gridDim.x) {
    const uint32_t b = P.lists[li];
    if ((P.plans[b].step_flags >> 8) == plan_flag) write_block_lds(P, b, smem);
  }
}

// ----------------------------------------------------- E3: HBM write pass
__global__ __launch_bounds__(64) void encode_large_kernel(EncodeParams P) {
  __shared__ uint32_t hlo[kE3HashChunk], hhi[kE3HashChunk];
  const int lane = threadIdx.x;
  const uint32_t count = P.list_count[0];
  for (uint32_t li = blockIdx.x; li < count; li += gridDim.x) {
    const uint32_t b = P.lists[li];
    const BlockPlan pl = P.plans[b];
    if ((pl.step_flags >> 8) != kPlanHuge) continue;
    const uint32_t step = pl.step_flags & 0xFF;
    const uint64_t dst_off = P.block_off[b], dst_end = P.block_off[b + 1];
    if (dst_end > P.out_cap) {
      if (lane == 0) P.status[b] = ST_OVERFLOW;
      continue;
    }
    const uint32_t s = P.starts[b], e = P.starts[b + 1], n = e - s;
    const uint32_t ri = is_index(P) ? 1 : P.ri;
    const uint32_t total = (uint32_t)(dst_end - dst_off);
    const uint32_t plen = total - kHdrLen;
    const uint64_t dabs = (uint64_t)(uintptr_t)P.out + dst_off;
    uint8_t* img = reinterpret_cast<uint8_t*>(dabs & ~15ULL);
    const uint32_t pad = (uint32_t)(dabs & 15);
    const uint32_t p0 = pad + kHdrLen;
    const uint32_t bin_off = pl.recs + 1;
    uint32_t carry = 0;
    for (uint32_t c = 0; c < n; c += kWave) {
      const uint32_t j = c + lane;
      const uint64_t i = (uint64_t)s + j;
      const bool head = j % ri == 0;
      ItemMeta m;
      RecordCopy rc;
      uint32_t rec = 0;
      if (j < n) {
        bool bad = false;
        m = load_item(P, i, bad);
        if (!is_index(P)) m.sh = P.shared[i];
        rec = (uint32_t)item_record_len(P, m, head);
      }
      const uint32_t incl = wave_incl_scan_u32(rec);
      const uint32_t roff = carry + incl - rec;
      if (j < n) {
        rc.issue(P, m, head, p0 + roff);
        rc.store(P, m, head, img);
        if (j % ri == 0) store_le(img, p0 + bin_off + (j / ri) * step, roff, step);
      }
      carry += wave_bcast_u32(incl, 63);
    }
    const uint32_t hash_off = pl.hash_w ? bin_off + pl.bin_len * step : 0;
    for (uint32_t base = 0; base < pl.hash_w; base += kE3HashChunk) {
      const uint32_t lim = min(kE3HashChunk, pl.hash_w - base);
      for (uint32_t k = lane; k < lim; k += kWave) { hlo[k] = 0xFFFFFFFFu; hhi[k] = 0; }
      __syncthreads();
      for (uint32_t j = lane; j < n; j += kWave) {
        const uint64_t i = (uint64_t)s + j;
        const uint64_t ko = P.it.key_off[i];
        const uint32_t bk = key_bucket(P, ko, (uint32_t)(P.it.key_off[i + 1] - ko), pl.hash_w);
        if (bk >= base && bk < base + lim) {
          atomicMin(&hlo[bk - base], j / ri);
          atomicMax(&hhi[bk - base], j / ri);
        }
      }
      __syncthreads();
      for (uint32_t k = lane; k < lim; k += kWave) img[p0 + hash_off + base + k] = (uint8_t)bucket_byte(hlo[k], hhi[k]);
      __syncthreads();
    }
    if (lane == 0) img[p0 + pl.recs] = kTrailerMarker;
    write_trailer_bytes(img, p0 + plen - kTrailerLen, ri, step, pl.bin_len, bin_off, pl.hash_w, hash_off, n);
    __threadfence();  // make this wave's HBM writes visible to its own re-reads below
    __syncthreads();
    uint64_t ck_lo, ck_hi;
    xxh3_128_wave(img, p0, plen, &kLongSecret, ck_lo, ck_hi);
    write_header_bytes(img, pad, P.type, ck_lo, ck_hi, plen);
    if (lane == 0) P.status[b] = ST_OK;
    __syncthreads();
  }
}

// Scan output: block offsets (low 40 bits of the prefix) and the list of the
// listed blocks (high bits = their running count).
struct EncodeOffOut {
  uint64_t* off;
  const uint64_t* sizes;
  uint32_t* list;
  uint32_t* count;
  uint64_t n;
  __device__ void operator()(uint64_t i, uint64_t prefix) const {
    off[i] = prefix & kOffMask;
    if (i < n && (sizes[i] & ~kOffMask)) list[prefix >> 40] = (uint32_t)i;
    if (i == n) *count = (uint32_t)(prefix >> 40);
  }
};

static size_t al256(size_t x) { return (x + 255) / 256 * 256; }

size_t encode_workspace_size(uint64_t n_items, uint32_t n_blocks) {
  return al256(n_items * 2) + al256((size_t)n_blocks * 8) + al256((size_t)n_blocks * sizeof(BlockPlan)) +
         al256((size_t)n_blocks * 4) + 256 + al256(scan_tiles(n_blocks) * 8);
}

uint64_t encode_bound(uint64_t n_items, uint32_t n_blocks, uint64_t key_bytes, uint64_t val_bytes,
                      const lsm_block_params* params) {
  const float ratio = params ? params->hash_ratio : 0.0f;
  uint64_t hash = 0;
  if (ratio > 0.0f) hash = (uint64_t)ceil((double)n_items * (double)ratio) + n_blocks;
  return 29ULL * n_items + key_bytes + val_bytes + 4ULL * n_items + hash +
         (uint64_t)n_blocks * (kHdrLen + 1 + kTrailerLen + 16) + 64;
}

hipError_t launch_encode(const lsm_items& items, const uint32_t* starts, uint32_t n_blocks,
                         const lsm_block_params& params, uint8_t* out, uint64_t out_cap, uint64_t* block_off,
                         int32_t* status, void* ws, hipStream_t st) {
  EncodeParams P;
  P.it = items;
  P.starts = starts;
  P.n_blocks = n_blocks;
  P.ri = params.block_type == 1 ? 1 : params.restart_interval;
  P.ratio = params.block_type == 1 ? 0.0f : params.hash_ratio;
  P.type = params.block_type;
  P.diag = params.reserved;
  P.out = out;
  P.out_cap = out_cap;
  P.block_off = block_off;
  P.status = status;
  uint8_t* w = (uint8_t*)ws;
  P.shared = (uint16_t*)w; w += al256(items.n_items * 2);
  P.sizes = (uint64_t*)w; w += al256((size_t)n_blocks * 8);
  P.plans = (BlockPlan*)w; w += al256((size_t)n_blocks * sizeof(BlockPlan));
  P.lists = (uint32_t*)w; w += al256((size_t)n_blocks * 4);
  P.list_count = (uint32_t*)w; w += 256;
  uint64_t* tiles = (uint64_t*)w;
  hipError_t e;
  hipLaunchKernelGGL(encode_sizes_kernel, dim3((n_blocks + 3) / 4), dim3(256), 0, st, P);
  if ((e = launch_excl_scan(P.sizes, n_blocks, tiles,
                            EncodeOffOut{block_off, P.sizes, P.lists, P.list_count, n_blocks}, st)) != hipSuccess)
    return e;
  static uint64_t attr_done = 0;
  if ((e = set_lds_attr((const void*)encode_write_list_kernel, kImgBig, &attr_done)) != hipSuccess) return e;
  hipLaunchKernelGGL(encode_write_kernel, dim3((n_blocks + kSmallWaves - 1) / kSmallWaves), dim3(kSmallWaves * kWave),
                     kSmallWaves * kImgSmall, st, P);
  hipLaunchKernelGGL(encode_write_list_kernel, dim3(2048), dim3(kWave), kImgMedium, st, P, kPlanMedium);
  hipLaunchKernelGGL(encode_write_list_kernel, dim3(512), dim3(kWave), kImgBig, st, P, kPlanBig);
  hipLaunchKernelGGL(encode_large_kernel, dim3(1024), dim3(64), 0, st, P);
  return hipGetLastError();
}

}  // namespace lsmgpu
