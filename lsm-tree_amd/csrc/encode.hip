// encode.hip — batched SST block encode on gfx950.
//
// Replaces, per block, DataBlock::encode_into / IndexBlock::encode_into
// (src/table/data_block/mod.rs:523-549, src/table/index_block/mod.rs:110-127,
// Encoder src/table/block/encoder.rs:84-164, Trailer trailer.rs:78-173) and
// Block::write_into (src/table/block/mod.rs:45-84, CompressionType::None):
// the payload xxh3_128 and the 33-byte header are fused into the same pass.
//
// Pipeline (all on one stream, DESIGN.md "Encode kernels"):
//   E1  encode_plan_kernel, thread per item over runs of 16 blocks: shared
//       prefix with the restart head (encoder.rs:140-143), record length,
//       LDS-atomic sums per block -> block size, binary-index step,
//       hash-index size, size class, key / value span starts.
//   S   device exclusive scan of block sizes -> d_block_off (packed output).
//   E2  encode_group_kernel: 4-wave workgroups write runs of consecutive
//       blocks in groups staged by LDS-DMA (key and value spans), thread per
//       record into an LDS image of the group's output span, binary index,
//       hash index (LDS min/max atomics reproduce the order-independent
//       FREE/idx/CONFLICT rule, hash_index/builder.rs:64-110), trailer, the
//       payload xxh3_128 split over the workgroup's 16 DPP rows in 1 KiB
//       units, headers, one coalesced 16 B/lane copy-out.
//   L   blocks that do not fit a group: listed 1-wave kernels (LDS image of
//       20 / 96 KiB) or E3 straight in HBM.
#include <hip/hip_runtime.h>

#include <math.h>

#include <algorithm>
#include <cstddef>
#include <type_traits>

#include "block_format.hpp"
#include "decode.hpp"
#include "encode.hpp"
#include "scan.hpp"
#include "fill.hpp"

namespace lsmgpu {

// Block classes: blocks that fit the group kernel's budget (group_fits) are
// written by encode_group_kernel; the others are listed by the size scan and
// written, by the LDS image they need (e2_need), by 1-wave workgroups with a
// 20 KiB (medium) or 96 KiB (big) image, or straight in HBM (E3, huge).
constexpr uint32_t kPlanHuge = 1, kPlanBad = 2, kPlanMedium = 4, kPlanBig = 8;
constexpr uint32_t kPlanHugeGpu = 16;  // a huge block the whole-GPU E3 path took over (not the one-workgroup E3)
constexpr uint32_t kImgMedium = 20 * 1024;
constexpr uint32_t kImgBig = 96 * 1024;
constexpr uint32_t kListBigWaves = 8;  // waves per listed big block
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
  uint32_t plan_bpw;  // blocks per plan workgroup (<= kPlanBlocks), see plan_blocks_per_wg
  uint8_t* out;
  uint64_t out_cap;
  uint64_t* block_off;
  int32_t* status;
  uint64_t* kspan;      // [n_blocks + 1] key_off of each block's first item (E1 -> E2 stage spans)
  uint64_t* vspan;      // [n_blocks + 1] val_off of each block's first item
  uint64_t* sizes;      // [n_blocks] block bytes (E1) -> exclusive scan -> block_off
  BlockPlan* plans;     // [n_blocks]
  uint32_t* lists;      // [n_blocks]: the listed blocks in block order (from the size scan)
  uint32_t* list_count; // [1]
  uint32_t* erec;       // [n_items] E1 -> E2, see kErec*
  uint16_t* hbucket;    // [n_items] E1 -> E2 (hash-index batches, when hb_valid): the key's bucket
                        // in its block (kNoBucket for blocks of >= kNeedHash buckets, never group-class)
  uint32_t hb_valid;
  uint32_t hb_sh;       // hbucket holds every non-head item's shared prefix length (E1p ran)
  uint32_t* hb_fix;     // [1] set by E1 when it left keys of more than 16 bytes (kNeedHash)
  unsigned long long* phase;  // diagnostic builds: per-phase cycle totals [16]
  uint32_t* pfirst;     // [n_blocks + 1] E1p: each block's first record prefix (low 32 bits); [n_blocks] the total
  uint32_t* e1p_flag;   // [1] E1p: the item_start array is not monotone
  uint64_t* wpart;      // [2 per wave of items] E1p: record totals of the blocks crossing a wave's ends
  uint8_t* huge_pool;   // workspace past encode_workspace_size (null: E3 one workgroup per block)
  uint64_t huge_pool_bytes;
  uint32_t huge_cap;    // huge-list entries the pool's layout provides
  uint32_t off32;       // it.key_off / it.val_off hold u32 offsets (lsm_encode_blocks32, lsm_items32)
};

__device__ __forceinline__ bool is_index(const EncodeParams& P) { return P.type == 1; }

// Key / value offset i: u64 arrays (lsm_items) or u32 arrays (lsm_items32: SURVEY 8(d)'s 4 + 4 B
// per item, arenas < 4 GiB).  kOW: the width in bytes when the kernel is instantiated for one
// (the hot plan and group kernels: straight-line loads), 0 = the batch-wide P.off32 at run time
// (a scalar branch per load site: the cold kernels).
template <int kOW = 0>
__device__ __forceinline__ bool off_w32(const EncodeParams& P) {
  return kOW == 4 || (kOW == 0 && P.off32);
}
template <int kOW = 0>
__device__ __forceinline__ uint64_t off_at(const EncodeParams& P, const uint64_t* a, uint64_t i) {
  return off_w32<kOW>(P) ? (uint64_t)gload(reinterpret_cast<const uint32_t*>(a), i) : gload(a, i);
}
template <int kOW = 0>
__device__ __forceinline__ uint64_t koff(const EncodeParams& P, uint64_t i) { return off_at<kOW>(P, P.it.key_off, i); }
template <int kOW = 0>
__device__ __forceinline__ uint64_t voff(const EncodeParams& P, uint64_t i) { return off_at<kOW>(P, P.it.val_off, i); }
// offset base + t with a wave-uniform base (SGPR pointer) and a per-lane t < 2^29 (32-bit byte offsets)
template <int kOW = 0>
__device__ __forceinline__ uint64_t off_rel(const EncodeParams& P, const uint64_t* a, uint64_t base, uint32_t t) {
  if (off_w32<kOW>(P))
    return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(reinterpret_cast<const uint32_t*>(a) + base) + 4u * t);
  return *reinterpret_cast<const uint64_t*>(reinterpret_cast<const uint8_t*>(a + base) + 8u * t);
}

// d_block_item_start[i] as E1 walks it: clamped to n_items, so no item field
// past the arenas is read (the reference takes &[InternalValue],
// data_block/mod.rs:523-549, so its block ranges are in bounds by type; the
// C ABI checks).  A block whose end is past n_items is rejected (ST_BAD_ARG).
__device__ __forceinline__ uint32_t clamped_start(const EncodeParams& P, uint32_t i) {
  const uint32_t v = P.starts[i];
  return (uint64_t)v > P.it.n_items ? (uint32_t)P.it.n_items : v;
}
__device__ __forceinline__ bool start_past_items(const EncodeParams& P, uint32_t i) {
  return (uint64_t)P.starts[i] > P.it.n_items;
}

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

// Destination pointers of the record writers: LDS images (lds8_t) or HBM
// (gbl8_t), explicit so that the stores compile to ds_write / global_store
// (a generic pointer gives flat stores, which also count on lgkmcnt: every
// later LDS wait then waits for the loads in flight too).
typedef __attribute__((address_space(3))) uint8_t lds8_t;
typedef __attribute__((address_space(1))) uint8_t gbl8_t;
__device__ __forceinline__ void st_u32(lds8_t* p, uint32_t v) { *(__attribute__((address_space(3))) uint32_t*)p = v; }
__device__ __forceinline__ void st_u32(gbl8_t* p, uint32_t v) { *(__attribute__((address_space(1))) uint32_t*)p = v; }
__device__ __forceinline__ void st_u32(uint8_t* p, uint32_t v) { *reinterpret_cast<uint32_t*>(p) = v; }
__device__ __forceinline__ lds8_t* as_lds(uint8_t* p) { return (lds8_t*)p; }
__device__ __forceinline__ gbl8_t* as_gbl(uint8_t* p) { return (gbl8_t*)p; }

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
  const __attribute__((address_space(1))) u32x4* W;
  uint32_t n, d, rel, nwin, h, tl, hb, tb;
  u32x4 w[K];
  __device__ __forceinline__ void load(const uint8_t* src, uint32_t n_, uint32_t d_) {
    const uint64_t a = (uint64_t)(uintptr_t)src;
    W = (const __attribute__((address_space(1))) u32x4*)(a & ~15ULL);
    n = n_;
    d = d_;
    rel = (uint32_t)(a & 15);
    nwin = n_ ? ((rel + n_ - 1) >> 4) + 1 : 0;
#pragma unroll
    for (int k = 0; k < K; ++k) w[k] = (uint32_t)k < nwin ? W[k] : u32x4{0, 0, 0, 0};
    h = min(n_, (4u - (d_ & 3u)) & 3u);
    tl = n_ > h ? (d_ + n_) & 3u : 0u;
    hb = tb = 0;
    const gbl8_t* gs = (const gbl8_t*)src;
    for (uint32_t k = 0; k < h; ++k) hb |= (uint32_t)gs[k] << (8 * k);
    for (uint32_t k = 0; k < tl; ++k) tb |= (uint32_t)gs[n_ - tl + k] << (8 * k);
  }
  template <class D>
  __device__ __forceinline__ void emit(D* dst, int wi, const u32x4& cw, uint32_t next0, int t0, uint32_t sh,
                                       uint32_t da, int qa, int qb) const {
    const uint32_t c[5] = {cw.x, cw.y, cw.z, cw.w, next0};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = 4 * wi + j - t0;
      if (q >= qa && q <= qb) st_u32(dst + da + 4 * q, alignbyte(c[j + 1], c[j], sh));
    }
  }
  template <class D>
  __device__ __forceinline__ void store(D* dst) const {
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
// 16-B copy-out store of the list / huge-block kernels (non-temporal: plain stores measured
// 0 to +2 % slower for the configs[4] classes, profiles/r06_experiments.txt; the group
// kernel's copy-out is plain)
__device__ __forceinline__ void copy_store16(u32x4* dst, const u32x4& v) { __builtin_nontemporal_store(v, dst); }

struct ItemMeta {
  uint64_t ko, vo, seq;
  uint32_t klen, vl, vt, sh;
  uint32_t e;   // E2 only: the plan's erec word
  uint32_t hb;  // E2 only: the plan's hash bucket (kNoBucket: none)
};
constexpr uint32_t kNoBucket = 0xFFFF;

constexpr uint32_t kNeedHash = 0xFFFE;  // E1 left this key (> 16 bytes) to encode_bucket_fixup_kernel

// An item's fields exactly as loaded (E2's one-group-ahead prefetch).  The
// offsets keep the width they were loaded with (RawItemT<4>: u32), so nothing
// widens them before cook_item consumes them: a zero-extension at the load
// made the compiler wait for the prefetched loads right there (the u32 group
// kernel ran 5 % slower with u64 fields here).
template <int kOW = 0, bool kIdx = false>
struct RawItemT {
  typedef typename std::conditional<kOW == 4, uint32_t, uint64_t>::type off_t;
  typedef typename std::conditional<kOW == 4 && !kIdx, uint32_t, uint64_t>::type voff_t;  // (index: handle offset)
  off_t ko, ko1;
  voff_t vo, vo1;  // (vo1: the index handle size for index blocks)
  uint64_t seq;
  uint32_t vt, e, hb;
};
typedef RawItemT<0> RawItem;

// Plain loads of item i's fields (no arithmetic, so no wait is forced here).
template <bool kIndex, int kOW = 0>
__device__ __forceinline__ RawItemT<kOW, kIndex> load_raw(const EncodeParams& P, uint64_t i) {
  RawItemT<kOW, kIndex> r;
  if (kOW == 4) {
    r.ko = gload(reinterpret_cast<const uint32_t*>(P.it.key_off), i);
    r.ko1 = gload(reinterpret_cast<const uint32_t*>(P.it.key_off), i + 1);
  } else {
    r.ko = koff<kOW>(P, i);
    r.ko1 = koff<kOW>(P, i + 1);
  }
  r.seq = P.it.seqno[i];
  r.e = 0;
  r.hb = kNoBucket;
  if (kIndex) {
    r.vo = P.it.handle_off[i];
    r.vo1 = P.it.handle_size[i];
    r.vt = 0;
  } else {
    if (kOW == 4) {
      r.vo = gload(reinterpret_cast<const uint32_t*>(P.it.val_off), i);
      r.vo1 = gload(reinterpret_cast<const uint32_t*>(P.it.val_off), i + 1);
    } else {
      r.vo = voff<kOW>(P, i);
      r.vo1 = voff<kOW>(P, i + 1);
    }
    r.vt = P.it.vtype[i];
  }
  return r;
}

// The same from a wave-uniform base item and a per-lane offset t < 2^29:
// base pointers in SGPRs and 32-bit byte offsets (one VGPR per address).
template <bool kIndex>
__device__ __forceinline__ RawItem load_raw_rel(const EncodeParams& P, uint64_t base, uint32_t t) {
  auto at64 = [&](const uint64_t* a, uint32_t k) {
    return *reinterpret_cast<const uint64_t*>(reinterpret_cast<const uint8_t*>(a + base) + 8u * k);
  };
  RawItem r;
  r.ko = off_rel(P, P.it.key_off, base, t);
  r.ko1 = off_rel(P, P.it.key_off, base, t + 1);
  r.seq = at64(P.it.seqno, t);
  r.e = 0;
  r.hb = kNoBucket;
  if (kIndex) {
    r.vo = at64(P.it.handle_off, t);
    r.vo1 = (P.it.handle_size + base)[t];
    r.vt = 0;
  } else {
    r.vo = off_rel(P, P.it.val_off, base, t);
    r.vo1 = off_rel(P, P.it.val_off, base, t + 1);
    r.vt = (P.it.vtype + base)[t];
  }
  return r;
}

// Derived fields of a raw item and the writer's argument checks (key length
// <= u16, a known value type, value length <= u32).
template <bool kIndex, class R>
__device__ __forceinline__ ItemMeta cook_item(const R& r, bool& bad) {
  ItemMeta m;
  const uint64_t kl = (uint64_t)r.ko1 - (uint64_t)r.ko;  // (widened first: a decreasing pair is bad at any width)
  if (kl > 0xFFFF) bad = true;
  m.ko = r.ko;
  m.klen = (uint32_t)min(kl, (uint64_t)0xFFFF);
  m.seq = r.seq;
  m.vo = r.vo;
  m.vt = r.vt;
  m.sh = 0;
  m.e = r.e;
  m.hb = r.hb;
  if (kIndex) {
    m.vl = (uint32_t)r.vo1;
  } else {
    const uint64_t vl = (uint64_t)r.vo1 - (uint64_t)r.vo;
    if (!valid_vtype(m.vt)) bad = true;
    if (!is_tombstone(m.vt) && vl > 0xFFFFFFFFULL) bad = true;
    m.vl = (uint32_t)vl;
  }
  return m;
}

template <int kOW = 0>
__device__ __forceinline__ ItemMeta load_item(const EncodeParams& P, uint64_t i, bool& bad) {
  ItemMeta m;
  m.ko = koff<kOW>(P, i);  // (global loads, not flat ones)
  const uint64_t kl = koff<kOW>(P, i + 1) - m.ko;
  if (kl > 0xFFFF) bad = true;
  m.klen = (uint32_t)min(kl, (uint64_t)0xFFFF);
  m.seq = gload(P.it.seqno, i);
  m.sh = 0;
  m.e = 0;
  if (is_index(P)) {
    m.vo = gload(P.it.handle_off, i);
    m.vl = gload(P.it.handle_size, i);
    m.vt = 0;
  } else {
    m.vo = voff<kOW>(P, i);
    const uint64_t vl = voff<kOW>(P, i + 1) - m.vo;
    m.vt = gload(P.it.vtype, i);
    if (!valid_vtype(m.vt)) bad = true;
    if (!is_tombstone(m.vt) && vl > 0xFFFFFFFFULL) bad = true;
    m.vl = (uint32_t)vl;
  }
  return m;
}

// Item j of the block starting at item s, with its shared prefix against the
// restart head (encoder.rs:140-143, util.rs:125-130).
template <int kOW = 0>
__device__ __forceinline__ ItemMeta load_item_lcp(const EncodeParams& P, uint32_t s, uint32_t j, uint32_t ri,
                                                  bool& bad) {
  const uint64_t i = (uint64_t)s + j;
  ItemMeta m = load_item<kOW>(P, i, bad);
  if (!is_index(P) && j % ri != 0) {
    const uint64_t h = (uint64_t)s + (j / ri) * ri;
    const uint64_t hko = koff<kOW>(P, h);
    const uint32_t hkl = (uint32_t)min(koff<kOW>(P, h + 1) - hko, (uint64_t)0xFFFF);
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
template <class D>
__device__ __forceinline__ uint32_t put_leb(D* dst, uint32_t pos, uint64_t v) {
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
  template <class D>
  __device__ __forceinline__ void store(const EncodeParams& P, const ItemMeta& m, bool head, D* dst) const {
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

template <class D>
__device__ __forceinline__ void store_le(D* dst, uint32_t pos, uint64_t v, uint32_t n) {
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

// The same header written by a lane quad (lane q of the quad: bytes
// [8q, 8q + 8), lane 0 also byte 32), every lane computing the 29-byte
// checksum itself.
__device__ __forceinline__ void write_header_quad(uint8_t* dst, uint32_t hp, uint32_t type, uint64_t ck_lo,
                                                  uint64_t ck_hi, uint32_t plen, int q) {
  const uint64_t w0 = 0x034D534CULL | ((uint64_t)type << 32) | (ck_lo << 40);
  const uint64_t w1 = (ck_lo >> 24) | (ck_hi << 40);
  const uint64_t w2 = (ck_hi >> 24) | ((uint64_t)plen << 40);
  const uint64_t w3 = ((uint64_t)plen >> 24) | ((uint64_t)plen << 8);
  auto r64 = [&](uint32_t o) -> uint64_t {  // LE u64 at byte o of w0..w3 (o <= 24)
    const uint32_t qq = o >> 3, sft = (o & 7) * 8;
    const uint64_t a = qq == 0 ? w0 : qq == 1 ? w1 : qq == 2 ? w2 : w3;
    const uint64_t b = qq == 0 ? w1 : qq == 1 ? w2 : qq == 2 ? w3 : 0;
    return sft ? (a >> sft) | (b << (64 - sft)) : a;
  };
  auto r8 = [&](uint32_t o) -> uint32_t { return (uint32_t)(r64(o) & 0xFF); };
  uint64_t hlo, hhi;
  xxh3_128_short(29, r8, r64, hlo, hhi);
  // bytes 29..32: the low 4 bytes of the header checksum
  const uint64_t w = q == 0 ? w0 : q == 1 ? w1 : q == 2 ? w2 : (w3 & 0xFFFFFFFFFFULL) | (hlo << 40);
  const uint32_t at = hp + 8 * q;
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i) dst[at + i] = (uint8_t)(w >> (8 * i));
  if (q == 0) dst[hp + 32] = (uint8_t)(hlo >> 24);
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
      copy_store16(reinterpret_cast<u32x4*>(gdst) + c, reinterpret_cast<const u32x4*>(img)[c]);
    } else {
      for (uint32_t k = max(lo, pad); k < min(hi, pad + total); ++k) gdst[k] = img[k];
    }
  }
  if (lane == 0) P.status[b] = ST_OK;
}

// Listed block b (any item count) assembled by one wave in the LDS image at
// `smem` (16-B aligned, at least e2_need bytes); shared prefixes and the plan
// come from the fused pass.
template <int kOW>
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
    const bool head = j % ri == 0;
    ItemMeta m;
    RecordCopy rc;
    uint32_t rec = 0;
    if (j < n) {
      bool bad = false;
      m = load_item_lcp<kOW>(P, s, j, ri, bad);
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

// The same block with every wave of a kLW-wave workgroup: items in chunks of
// kLW * 64 (workgroup scan), then marker / hash-index bytes / trailer, the
// payload xxh3_128 (per-KiB contributions on every wave into `contrib`, the
// scramble chain and the merge on wave 0), the header and the copy-out.  One
// wave per 20-96 KiB block ran the 64 KiB classes at 0.18 TB/s.
template <uint32_t kLW, int kOW>
__device__ __forceinline__ void write_block_lds_mw(const EncodeParams& P, uint32_t b, uint8_t* smem, uint32_t* psum,
                                                   uint64_t* contrib) {
  constexpr uint32_t kT = kLW * kWave;
  const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1);
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const uint32_t s = P.starts[b], e = P.starts[b + 1];
  const uint64_t dst_off = P.block_off[b], dst_end = P.block_off[b + 1];
  const BlockPlan pl = P.plans[b];
  const uint32_t step = pl.step_flags & 0xFF;
  if (dst_end > P.out_cap) {
    if (tid == 0) P.status[b] = ST_OVERFLOW;
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
  for (uint32_t k = tid; k < pl.hash_w; k += kT) {
    hlo[k] = 0xFFFFFFFFu;
    hhi[k] = 0;
  }
  __syncthreads();
  const uint32_t p0 = pad + kHdrLen;
  const uint32_t bin_off = pl.recs + 1;
  uint32_t carry = 0;
  for (uint32_t c = 0; c < n; c += kT) {
    const uint32_t j = c + tid;
    const bool head = j % ri == 0;
    ItemMeta m;
    RecordCopy rc;
    uint32_t rec = 0;
    if (j < n) {
      bool bad = false;
      m = load_item_lcp<kOW>(P, s, j, ri, bad);
      rec = (uint32_t)item_record_len(P, m, head);
    }
    const uint32_t incl = wave_incl_scan_u32(rec);
    if (lane == kWave - 1) psum[wave] = incl;
    __syncthreads();
    uint32_t wbase = 0, tot = 0;
    for (uint32_t w = 0; w < kLW; ++w) {
      const uint32_t v = psum[w];
      wbase += w < wave ? v : 0u;
      tot += v;
    }
    const uint32_t roff = carry + wbase + incl - rec;
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
    carry += tot;
    __syncthreads();  // (psum is rewritten by the next chunk; the votes are complete)
  }
  const uint32_t plen = total - kHdrLen;
  const uint32_t hash_off = pl.hash_w ? bin_off + pl.bin_len * step : 0;
  if (tid == 0) img[p0 + pl.recs] = kTrailerMarker;
  for (uint32_t k = tid; k < pl.hash_w; k += kT) img[p0 + hash_off + k] = (uint8_t)bucket_byte(hlo[k], hhi[k]);
  if (wave == 0) write_trailer_bytes(img, p0 + plen - kTrailerLen, ri, step, pl.bin_len, bin_off, pl.hash_w, hash_off, n);
  __syncthreads();
  uint64_t lo = 0, hi = 0;
  if (plen > 240) {
    const int q = lane & 3;
    uint64_t a0, a1;
    xxh3_acc_init(q, a0, a1);
    const uint64_t scr0 = kLongSecret.acc[16 + 2 * q], scr1 = kLongSecret.acc[16 + 2 * q + 1];
    const uint32_t nbk = (plen - 1) / 1024;
    for (uint32_t n0 = 0; n0 < nbk; n0 += 64) {
      const uint32_t n1 = min(nbk, n0 + 64);
      xxh3_kib_contribs(img, p0 + 1024 * n0, (n1 - n0) * 1024 + 1, &kLongSecret, contrib, wave, kLW);
      __syncthreads();
      if (wave == 0)
        for (uint32_t k = 0; k < n1 - n0; ++k) {
          a0 = xxh3_scr(a0, contrib[8 * k + 2 * q], scr0);
          a1 = xxh3_scr(a1, contrib[8 * k + 2 * q + 1], scr1);
        }
      __syncthreads();
    }
    if (wave == 0) xxh3_wave_tail_merge(img, p0, plen, &kLongSecret, a0, a1, lo, hi);
  } else if (wave == 0) {
    xxh3_128_wave(img, p0, plen, &kLongSecret, lo, hi);
  }
  if (wave == 0) write_header_bytes(img, pad, P.type, lo, hi, plen);
  __syncthreads();
  uint8_t* gdst = reinterpret_cast<uint8_t*>(dabs & ~15ULL);
  const uint32_t chunks = (pad + total + 15) >> 4;
  for (uint32_t c = tid; c < chunks; c += kT) {
    const uint32_t clo = c * 16, chi = clo + 16;
    if (clo >= pad && chi <= pad + total) {
      copy_store16(reinterpret_cast<u32x4*>(gdst) + c, reinterpret_cast<const u32x4*>(img)[c]);
    } else {
      for (uint32_t k = max(clo, pad); k < min(chi, pad + total); ++k) gdst[k] = img[k];
    }
  }
  if (tid == 0) P.status[b] = ST_OK;
  __syncthreads();  // (the next block reuses the image)
}

// Per-item word from E1 to E2 (read for group-class blocks, whose payload is
// < 32 KiB and whose items are < 2^16): bits 0-14 the record's offset in the
// block payload, bit 15 restart head, bits 16-31 the restart index (heads)
// or the shared-prefix length (keys are < 2^16 bytes).
constexpr uint32_t kErecHead = 0x8000u;

// Group write kernel (E2) budget, see encode_group_kernel.
constexpr uint32_t kGWaves = 4, kGThreads = kGWaves * kWave;
constexpr uint32_t kGRun = 32;          // blocks per workgroup (<= 63: one lane each)
constexpr uint32_t kGRunFused = 32;  // the same with the fused run-level plan (48 / 63: r06_experiments ab6h)
constexpr uint64_t kFusedAutoItems = 128;  // items per block from which the fused plan is taken
static_assert(kGRunFused <= 63, "one lane per block and one for the run's end");
constexpr uint32_t kGBlocks = 16;    // blocks per group
constexpr uint32_t kGItems = kGThreads;        // items per group (one thread each)
constexpr uint32_t kGSlack = 48;               // readable bytes past each staged span
// group LDS budget (four configs[1] blocks by default)
constexpr uint32_t kGKeys = 4096, kGVals = 14400, kGImg = 15872;
constexpr uint32_t kGUnits = kGImg / 1024 + kGBlocks + 1;  // hash units per group
constexpr uint32_t kGUnion = 4096;      // hash votes | hash contributions
constexpr uint32_t kGHash = kGUnion / 8;       // vote pairs
static_assert(kGUnits * 64 <= kGUnion, "hash contributions");
static_assert((kGUnits + 4) * 64 <= kGUnion, "the chain's batched reads stay inside L.uni");


__device__ __host__ __forceinline__ bool group_fits(uint64_t n, uint64_t kspan, uint64_t vspan, uint64_t total,
                                                    uint32_t hash_w) {
  return n <= kGItems && kspan + 15 <= kGKeys && vspan + 15 <= kGVals && total + 15 <= kGImg && hash_w <= kGHash;
}


// ---------------------------------------------------------------- E1: plan
// A 256-thread workgroup owns kPlanBlocks consecutive blocks and walks their
// items (contiguous) in chunks of 1024, four consecutive items per thread, so
// each wave has four items' loads in flight at once.  Per chunk:
//   1. item fields (key / value offsets, seqno, type); key offsets to LDS;
//   2. the shared prefix with the restart head (encoder.rs:140-143,
//      util.rs:125-130): the head's key offset from LDS (global only for a
//      head before the chunk), both keys' first 16 bytes as two aligned 16-B
//      loads each, all four items' loads issued together (longer equal
//      prefixes continue in lcp_global);
//   3. record lengths, a workgroup scan in item order -> each record's offset
//      in its block, kept for E2 in erec.
// Per block: size, binary-index step, hash-index size, size class, and the
// key / value span starts E2 stages.
// blocks per workgroup: longer-lived workgroups (16 -> 128: 0.80 -> 0.68 ms per 1 M blocks)
constexpr uint32_t kPlanBlocks = 128;
static_assert(kPlanBlocks <= 255, "thread nb loads the run's end: nb < 256 threads");
constexpr uint32_t kPlanPer = 2;          // consecutive items per thread
constexpr uint32_t kPlanChunk = 256 * kPlanPer;      // items per chunk

// 16 bytes at p (global, any alignment): one unaligned 16-B load (the arenas are
// padded).  Two aligned loads and a funnel shift issued twice the loads and ~10 VALU
// more per window, and held 20 more VGPRs in the plan kernel (113 -> 93, u32 offsets):
// 1-1.5 % faster encodes (profiles/r06_experiments.txt, ab6k).
__device__ __forceinline__ Win16 gwin16(const uint8_t* p) {
  Win16 r;
  __builtin_memcpy(&r, p, 16);
  return r;
}
__device__ __forceinline__ Win16 gwin16a(const uint8_t* p) { return gwin16(p); }

// Shared prefix past an equal first 16 bytes: 16 bytes per step (rare: long
// common key prefixes; kept narrow so the common path's registers stay low).
__device__ __noinline__
uint32_t lcp_tail(const uint8_t* keys, uint64_t a, uint64_t b, uint32_t n) {
  for (uint32_t k = 16; k < n; k += 16) {
    const Win16 wa = gwin16(keys + a + k), wb = gwin16(keys + b + k);
    const uint64_t x0 = wa.lo ^ wb.lo, x1 = wa.hi ^ wb.hi;
    if (x0) return min(n, k + (uint32_t)(__builtin_ctzll(x0) >> 3));
    if (x1) return min(n, k + 8 + (uint32_t)(__builtin_ctzll(x1) >> 3));
  }
  return n;
}

template <bool kIndex>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1))) void encode_plan_kernel(EncodeParams P) {
  __shared__ uint32_t bst[kPlanBlocks + 1];
  __shared__ unsigned long long bfirst[kPlanBlocks], bend[kPlanBlocks], lhead[kPlanBlocks];
  __shared__ unsigned long long psum[4];
  __shared__ uint32_t badf[kPlanBlocks];
  __shared__ uint32_t mono;
  __shared__ unsigned long long kos[kPlanChunk + 1];  // key offsets of the chunk's items (+ the next)
  const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  const uint32_t b0 = blockIdx.x * P.plan_bpw;
  const uint32_t nb = min(P.plan_bpw, P.n_blocks - b0);
  if (tid <= nb) bst[tid] = clamped_start(P, b0 + tid);
  if (tid < nb) {
    bfirst[tid] = bend[tid] = lhead[tid] = 0;
    badf[tid] = 0;
  }
  if (tid == 0) mono = 1;
  __syncthreads();
  if (tid < nb && bst[tid + 1] < bst[tid]) mono = 0;  // (benign race: every writer stores 0)
  __syncthreads();
  const uint32_t ri = kIndex ? 1 : P.ri;
  constexpr bool index = kIndex;
  // a non-monotone item_start run is a caller error: its blocks are rejected below
  // (wave-uniform: chunk bases stay in SGPRs, so item loads take the saddr form)
  const uint64_t i_begin = (uint32_t)__builtin_amdgcn_readfirstlane(bst[0]);
  const uint64_t i_end = (uint32_t)__builtin_amdgcn_readfirstlane(mono ? bst[nb] : bst[0]);
  uint64_t carry = 0;
  for (uint64_t base = i_begin; base < i_end; base += kPlanChunk) {
    const uint64_t i0 = base + kPlanPer * tid;
    // ---- 1. item fields, block of each item
    RawItem raw[kPlanPer];
#pragma unroll
    for (uint32_t q = 0; q < kPlanPer; ++q)
      raw[q] = load_raw_rel<kIndex>(P, base, (uint32_t)min(i0 + q, i_end - 1) - (uint32_t)base);
    ItemMeta m[kPlanPer];
    uint32_t jq[kPlanPer], jjq[kPlanPer];
    uint32_t j = 0;
    if (i0 < i_end) {
      uint32_t lo = 0, hi = nb;  // block j: bst[j] <= i0 < bst[j + 1]
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (bst[mid] <= i0) lo = mid;
        else hi = mid;
      }
      j = lo;
    }
#pragma unroll
    for (uint32_t q = 0; q < kPlanPer; ++q) {
      const uint64_t i = i0 + q;
      jq[q] = jjq[q] = 0;
      if (i < i_end) {
        while (j + 1 < nb && bst[j + 1] <= i) ++j;
        jq[q] = j;
        jjq[q] = (uint32_t)(i - bst[j]);
      }
    }
#pragma unroll
    for (uint32_t q = 0; q < kPlanPer; ++q) {
      bool bad = false;
      m[q] = cook_item<kIndex>(raw[q], bad);
      if (i0 + q < i_end) {
        if (bad) atomicOr(&badf[jq[q]], 1u);
        kos[kPlanPer * tid + q] = m[q].ko;
      }
    }
    __syncthreads();
    // ---- 2. shared prefix with the restart head
    if (!index) {
      Win16 wa[kPlanPer], wb[kPlanPer];
      uint32_t nq[kPlanPer];
      uint64_t hq[kPlanPer];
#pragma unroll
      for (uint32_t q = 0; q < kPlanPer; ++q) {
        const uint64_t i = i0 + q;
        nq[q] = 0;
        hq[q] = 0;
        if (i < i_end && jjq[q] % ri != 0) {
          const uint64_t h = i - jjq[q] % ri;  // restart head of item i
          const uint64_t hko = h >= base ? kos[h - base] : koff(P, h);
          const uint64_t hke = h + 1 >= base ? kos[h + 1 - base] : koff(P, h + 1);
          const uint32_t hkl = (uint32_t)min(hke - hko, (uint64_t)0xFFFF);
          nq[q] = min(hkl, m[q].klen);
          hq[q] = hko;
          wa[q] = gwin16(P.it.keys + hko);
          wb[q] = gwin16(P.it.keys + m[q].ko);
        }
      }
#pragma unroll
      for (uint32_t q = 0; q < kPlanPer; ++q) {
        if (!nq[q]) continue;
        const uint64_t x0 = wa[q].lo ^ wb[q].lo, x1 = wa[q].hi ^ wb[q].hi;
        const uint32_t n = nq[q];
        uint32_t sh;
        if (x0) sh = min(n, (uint32_t)(__builtin_ctzll(x0) >> 3));
        else if (x1) sh = min(n, 8 + (uint32_t)(__builtin_ctzll(x1) >> 3));
        else sh = n <= 16 ? n : lcp_tail(P.it.keys, hq[q], m[q].ko, n);
        m[q].sh = sh;
      }
    }
    // ---- 3. record lengths, workgroup scan in item order
    uint64_t rec[kPlanPer], tsum = 0;
#pragma unroll
    for (uint32_t q = 0; q < kPlanPer; ++q) {
      rec[q] = 0;
      if (i0 + q < i_end) rec[q] = item_record_len(P, m[q], jjq[q] % ri == 0);
      tsum += rec[q];
    }
    const uint64_t incl = wave_incl_scan_u64(tsum);
    if (lane == kWave - 1) psum[wave] = incl;
    __syncthreads();
    uint64_t wbase = 0, ptot = 0;
#pragma unroll
    for (uint32_t w = 0; w < 4; ++w) {
      const uint64_t v = psum[w];
      wbase += w < wave ? v : 0;
      ptot += v;
    }
    uint64_t ex = carry + wbase + incl - tsum;
    uint64_t exq[kPlanPer];
#pragma unroll
    for (uint32_t q = 0; q < kPlanPer; ++q) {
      exq[q] = ex;
      if (i0 + q < i_end) {
        const uint32_t jb = jq[q], jj = jjq[q], ridx = jj / ri;
        const uint32_t n = bst[jb + 1] - bst[jb];
        if (jj == 0) bfirst[jb] = ex;
        if (jj + 1 == n) bend[jb] = ex + rec[q];
        if (jj == ridx * ri && ridx == (n - 1) / ri) lhead[jb] = ex;
      }
      ex += rec[q];
    }
    __syncthreads();  // (also orders this chunk's psum / kos reads before the next chunk's writes)
#pragma unroll
    for (uint32_t q = 0; q < kPlanPer; ++q) {
      if (i0 + q < i_end) {
        const uint32_t jj = jjq[q], ridx = jj / ri;
        const bool head = jj == ridx * ri;
        const uint64_t roff = exq[q] - bfirst[jq[q]];
        const uint32_t x = head ? ridx : m[q].sh;
        // blocks of more than kGItems items are never group-class: their items
        // keep the whole 32-bit record offset, for E3
        P.erec[i0 + q] = bst[jq[q] + 1] - bst[jq[q]] > kGItems ? (uint32_t)min(roff, (uint64_t)0xFFFFFFFFu)
                                     : (uint32_t)min(roff, (uint64_t)0x7FFF) | (head ? kErecHead : 0u) |
                                           (min(x, 0xFFFFu) << 16);
      }
    }
    carry += ptot;
  }
  __syncthreads();
  if (tid >= nb) return;
  const uint32_t b = b0 + tid, s = bst[tid], e = bst[tid + 1];
  bool bad = !mono || e <= s || badf[tid] || start_past_items(P, b + 1);
  const uint32_t n = bad ? 0 : e - s;
  const uint64_t recs = bad ? 0 : bend[tid] - bfirst[tid], last_head = bad ? 0 : lhead[tid] - bfirst[tid];
  const uint32_t bin_len = n ? (n + ri - 1) / ri : 0;
  const uint32_t step = last_head <= 0xFFFF ? 2 : 4;
  const uint32_t buckets = kIndex ? 0 : bucket_count(n, P.ratio);
  const uint32_t hash_w = (buckets > 0 && bin_len <= kHashMaxPointers) ? buckets : 0;
  const uint64_t total = kHdrLen + recs + 1 + (uint64_t)bin_len * step + hash_w + kTrailerLen;
  if (recs > 0xFFFFFFF0ULL || total > 0xFFFFFF00ULL) bad = true;
  const uint64_t ks = koff(P, s), ke = koff(P, e);
  const uint64_t vs = kIndex ? 0 : voff(P, s), ve = kIndex ? 0 : voff(P, e);
  uint32_t flags = 0;
  if (bad) {
    flags = kPlanBad;
    P.status[b] = ST_BAD_ARG;
  } else if (!group_fits(n, ke - ks, ve - vs, total, hash_w)) {
    const uint64_t need = e2_need(total, hash_w);
    flags = need <= kImgMedium ? kPlanMedium : need <= kImgBig ? kPlanBig : kPlanHuge;
  }
  P.plans[b] = BlockPlan{(uint32_t)recs, bin_len, hash_w, step | (flags << 8)};
  // bits 40.. count the listed (not group) blocks: the size scan numbers them
  P.sizes[b] = (bad ? 0 : total) | ((flags & (kPlanMedium | kPlanBig | kPlanHuge)) ? kListedOne : 0);
  P.kspan[b] = ks;
  P.vspan[b] = vs;
  if (b + 1 == P.n_blocks) {
    P.kspan[b + 1] = ke;
    P.vspan[b + 1] = ve;
  }
}

// ------------------------------------- E1 for data blocks: wave-level runs
// The outputs of encode_plan_kernel<false> without workgroup barriers in the
// item loop: the workgroup's blocks are split among its four waves by item
// count (whole blocks each), and every wave walks its own items in steps of
// 128 (two consecutive items per lane).  Record offsets come from a wave scan
// plus a carry (a block never spans two waves); the shared prefix with the
// restart head (encoder.rs:140-143, util.rs:125-130) takes the head's key
// offset from the step's LDS copy, or for a head before the step from the
// carried last head; and the next step's item fields are loaded while this
// step's key windows are in flight.
constexpr uint32_t kPW = 2;  // consecutive items per lane
constexpr uint32_t kPWStep = kPW * kWave;
struct PlanWaveLds {
  uint32_t bst[kPlanBlocks + 1];
  uint32_t badf[kPlanBlocks];
  uint32_t wcut[5];
  uint32_t mono;
  unsigned long long bfirst[kPlanBlocks], bend[kPlanBlocks], lhead[kPlanBlocks];
  unsigned long long kos[4][kPWStep];
  uint32_t kls[4][kPWStep];
  Win16 kwin[4][kPWStep];  // each item's first 16 key bytes
};

// The plan of blocks [b0, b0 + nb) on one 256-thread workgroup (all threads call it).
// kFused (encode_group_kernel's run-level plan): each block's plan and size also go to
// fplan / fsize in LDS (thread j = block b0 + j), and P.sizes is not written (the fused
// kernel keeps its look-back words there).
template <bool kBkt, int kOW, bool kFused>
__device__ __forceinline__ void plan_wave_run(const EncodeParams& P, uint32_t b0, uint32_t nb, PlanWaveLds& S,
                                              BlockPlan* fplan, uint64_t* fsize) {
  uint32_t* const bst = S.bst;
  unsigned long long* const bfirst = S.bfirst;
  unsigned long long* const bend = S.bend;
  unsigned long long* const lhead = S.lhead;
  auto& kos = S.kos;
  auto& kls = S.kls;
  auto& kwin = S.kwin;
  uint32_t* const badf = S.badf;
  uint32_t* const wcut = S.wcut;
  uint32_t& mono = S.mono;
  const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1);
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  if (tid <= nb) bst[tid] = clamped_start(P, b0 + tid);
  if (tid < nb) {
    bfirst[tid] = bend[tid] = lhead[tid] = 0;
    badf[tid] = 0;
  }
  if (tid == 0) mono = 1;
  __syncthreads();
  if (tid < nb && bst[tid + 1] < bst[tid]) mono = 0;  // (benign race: every writer stores 0)
  if (tid <= 4) {  // wave t's first block: the first at or after a quarter of the items
    const uint32_t target = bst[0] + (uint32_t)(((uint64_t)(bst[nb] - bst[0]) * tid) / 4);
    uint32_t lo = 0, hi = nb;  // first j with bst[j] >= target (bst[nb] >= target)
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (bst[mid] >= target) hi = mid;
      else lo = mid + 1;
    }
    wcut[tid] = tid == 4 ? nb : lo;
  }
  __syncthreads();
  const uint32_t ri = P.ri;
  const uint32_t jlo = __builtin_amdgcn_readfirstlane(wcut[wave]);
  const uint32_t jhi = __builtin_amdgcn_readfirstlane(mono ? wcut[wave + 1] : wcut[wave]);
  const uint32_t ia = __builtin_amdgcn_readfirstlane(bst[jlo]);
  const uint32_t ie = __builtin_amdgcn_readfirstlane(bst[jhi]);
  unsigned long long* wkos = kos[wave];
  uint32_t* wkls = kls[wave];
  Win16* wkwin = kwin[wave];
  // a lane's two consecutive items: key / value offsets [t, t + 3), seqnos and types [t, t + 2)
  struct StepRaw {  // (offsets at their loaded width: see RawItemT)
    typename RawItemT<kOW>::off_t ko[kPW + 1], vo[kPW + 1];
    uint64_t seq[kPW];
    uint32_t vt[kPW];
  };
  auto load_step = [&](uint32_t base, StepRaw& r) {
    // (items past the run are clamped to its last one and ignored; offsets index up to ie)
    const uint32_t n = ie - base, t = min(kPW * lane, n - 1);
    auto at64 = [&](const uint64_t* a, uint32_t k) {
      return *reinterpret_cast<const uint64_t*>(reinterpret_cast<const uint8_t*>(a + base) + 8u * k);
    };
#pragma unroll
    for (uint32_t q = 0; q <= kPW; ++q) {
      r.ko[q] = (typename RawItemT<kOW>::off_t)off_rel<kOW>(P, P.it.key_off, base, min(t + q, n));
      r.vo[q] = (typename RawItemT<kOW>::off_t)off_rel<kOW>(P, P.it.val_off, base, min(t + q, n));
    }
#pragma unroll
    for (uint32_t q = 0; q < kPW; ++q) {
      r.seq[q] = at64(P.it.seqno, min(t + q, n - 1));
      r.vt[q] = (P.it.vtype + base)[min(t + q, n - 1)];
    }
  };
  StepRaw raw;
  if (ia < ie) load_step(ia, raw);
  uint64_t carry = 0;     // record bytes of this wave's items before the step
  uint64_t hk_ko = 0;     // the last restart head of the previous step: key offset, key length
  uint32_t hk_kl = 0;
  Win16 hk_win{0, 0};
  for (uint32_t base = ia; base < ie; base += kPWStep) {
    const uint32_t t0 = kPW * lane;
    ItemMeta m[kPW];
    uint32_t jq[kPW], jjq[kPW];
    bool ok[kPW];
    uint32_t j = jlo;
    {
      uint32_t lo = jlo, hi = jhi;  // block j: bst[j] <= base + t0 < bst[j + 1]
      const uint32_t i0 = min(base + t0, ie - 1);
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (bst[mid] <= i0) lo = mid;
        else hi = mid;
      }
      j = lo;
    }
#pragma unroll
    for (uint32_t q = 0; q < kPW; ++q) {
      const uint32_t i = base + t0 + q;
      ok[q] = i < ie;
      while (j + 1 < jhi && bst[j + 1] <= i) ++j;
      jq[q] = j;
      jjq[q] = ok[q] ? i - bst[j] : 0;
      bool bad = false;
      RawItem r;
      r.ko = raw.ko[q];
      r.ko1 = raw.ko[q + 1];
      r.vo = raw.vo[q];
      r.vo1 = raw.vo[q + 1];
      r.seq = raw.seq[q];
      r.vt = raw.vt[q];
      r.e = 0;
      r.hb = kNoBucket;
      m[q] = cook_item<false>(r, bad);
      if (ok[q] && bad) atomicOr(&badf[j], 1u);
      wkos[t0 + q] = m[q].ko;
      wkls[t0 + q] = m[q].klen;
    }
    // the next step's item fields, into the registers just consumed (no copy at the
    // step's end, which made the compiler wait for them there), in flight under this
    // step; issued before the key windows, which the step waits for
    if (base + kPWStep < ie) load_step(base + kPWStep, raw);
    // ---- shared prefix with the restart head: every item loads its own first 16
    // key bytes once; the others of its interval read the head's from LDS
    Win16 wa[kPW], wb[kPW];
#pragma unroll
    for (uint32_t q = 0; q < kPW; ++q) wb[q] = gwin16a(P.it.keys + m[q].ko);
#pragma unroll
    for (uint32_t q = 0; q < kPW; ++q) wkwin[t0 + q] = wb[q];
    if (kBkt) {  // hash-index batches: each key's bucket in its block, for E2 (keys of <= 16
                 // bytes from their window here, longer ones by encode_bucket_fixup_kernel)
#pragma unroll
      for (uint32_t q = 0; q < kPW; ++q) {
        if (!ok[q]) continue;
        const uint32_t n = bst[jq[q] + 1] - bst[jq[q]];
        const uint32_t buckets = bucket_count(n, P.ratio);
        const uint32_t hw = (buckets > 0 && (n + ri - 1) / ri <= kHashMaxPointers) ? buckets : 0;
        uint32_t hb = kNoBucket;
        if (hw && hw < kNeedHash) {  // (group-class blocks have at most kGHash buckets)
          if (m[q].klen <= 16)
            hb = (uint32_t)(xxh3_64_le16(m[q].klen, WinReader8{wb[q].lo, wb[q].hi},
                                         WinReader64{wb[q].lo, wb[q].hi}) % hw);
          else
            hb = kNeedHash, P.hb_fix[0] = 1;
        }
        P.hbucket[(uint64_t)base + t0 + q] = (uint16_t)hb;
      }
    }
    wave_lds_sync();
    uint32_t nq[kPW];
    uint64_t hq[kPW];
#pragma unroll
    for (uint32_t q = 0; q < kPW; ++q) {
      nq[q] = 0;
      hq[q] = 0;
      wa[q] = wb[q];
      if (ok[q] && jjq[q] % ri != 0) {
        const uint32_t h = base + t0 + q - jjq[q] % ri;
        const bool in = h >= base;
        const uint64_t hko = in ? (uint64_t)wkos[h - base] : hk_ko;
        const uint32_t hkl = in ? wkls[h - base] : hk_kl;
        nq[q] = min(hkl, m[q].klen);
        hq[q] = hko;
        wa[q] = in ? wkwin[h - base] : hk_win;
      }
    }
#pragma unroll
    for (uint32_t q = 0; q < kPW; ++q) {
      if (!nq[q]) continue;
      const uint64_t x0 = wa[q].lo ^ wb[q].lo, x1 = wa[q].hi ^ wb[q].hi;
      const uint32_t n = nq[q];
      uint32_t sh;
      if (x0) sh = min(n, (uint32_t)(__builtin_ctzll(x0) >> 3));
      else if (x1) sh = min(n, 8 + (uint32_t)(__builtin_ctzll(x1) >> 3));
      else sh = n <= 16 ? n : lcp_tail(P.it.keys, hq[q], m[q].ko, n);
      m[q].sh = sh;
    }
    // ---- record lengths, wave scan (a block never spans two waves)
    uint64_t rec[kPW], tsum = 0;
#pragma unroll
    for (uint32_t q = 0; q < kPW; ++q) {
      rec[q] = ok[q] ? item_record_len(P, m[q], jjq[q] % ri == 0) : 0;
      tsum += rec[q];
    }
    const uint64_t incl = wave_incl_scan_u64(tsum);
    uint64_t ex = carry + incl - tsum;
    uint64_t exq[kPW];
#pragma unroll
    for (uint32_t q = 0; q < kPW; ++q) {
      exq[q] = ex;
      if (ok[q]) {
        const uint32_t jb = jq[q], jj = jjq[q], ridx = jj / ri;
        const uint32_t n = bst[jb + 1] - bst[jb];
        if (jj == 0) bfirst[jb] = ex;
        if (jj + 1 == n) bend[jb] = ex + rec[q];
        if (jj == ridx * ri && ridx == (n - 1) / ri) lhead[jb] = ex;
      }
      ex += rec[q];
    }
    wave_lds_sync();
#pragma unroll
    for (uint32_t q = 0; q < kPW; ++q) {
      if (ok[q]) {
        const uint32_t jj = jjq[q], ridx = jj / ri;
        const bool head = jj == ridx * ri;
        const uint64_t roff = exq[q] - bfirst[jq[q]];
        const uint32_t x = head ? ridx : m[q].sh;
        // blocks of more than kGItems items are never group-class: their items
        // keep the whole 32-bit record offset, for E3
        P.erec[(uint64_t)base + t0 + q] =
            bst[jq[q] + 1] - bst[jq[q]] > kGItems
                ? (uint32_t)min(roff, (uint64_t)0xFFFFFFFFu)
                : (uint32_t)min(roff, (uint64_t)0x7FFF) | (head ? kErecHead : 0u) | (min(x, 0xFFFFu) << 16);
      }
    }
    carry += wave_bcast_u64(incl, kWave - 1);
    {  // the restart head of the step's last item, for the next step's first items
      const uint32_t last = min(ie, base + kPWStep) - 1, ll = (last - base) / kPW, lq = (last - base) % kPW;
      uint32_t jsel = jjq[0];
#pragma unroll
      for (uint32_t q = 1; q < kPW; ++q) jsel = lq == q ? jjq[q] : jsel;
      const uint32_t jjl = __builtin_amdgcn_readlane((int)jsel, (int)ll);
      const uint32_t h = last - jjl % ri;
      if (h >= base) {
        hk_ko = wkos[h - base];
        hk_kl = wkls[h - base];
        hk_win = wkwin[h - base];
      }
    }
    wave_lds_sync();  // (the next step rewrites kos / kls)
  }
  __syncthreads();
  if (tid >= nb) return;
  const uint32_t b = b0 + tid, s = bst[tid], e = bst[tid + 1];
  bool bad = !mono || e <= s || badf[tid] || start_past_items(P, b + 1);
  const uint32_t n = bad ? 0 : e - s;
  const uint64_t recs = bad ? 0 : bend[tid] - bfirst[tid], last_head = bad ? 0 : lhead[tid] - bfirst[tid];
  const uint32_t bin_len = n ? (n + ri - 1) / ri : 0;
  const uint32_t step = last_head <= 0xFFFF ? 2 : 4;
  const uint32_t buckets = bucket_count(n, P.ratio);
  const uint32_t hash_w = (buckets > 0 && bin_len <= kHashMaxPointers) ? buckets : 0;
  const uint64_t total = kHdrLen + recs + 1 + (uint64_t)bin_len * step + hash_w + kTrailerLen;
  if (recs > 0xFFFFFFF0ULL || total > 0xFFFFFF00ULL) bad = true;
  const uint64_t ks = koff<kOW>(P, s), ke = koff<kOW>(P, e);
  const uint64_t vs = voff<kOW>(P, s), ve = voff<kOW>(P, e);
  uint32_t flags = 0;
  if (bad) {
    flags = kPlanBad;
    P.status[b] = ST_BAD_ARG;
  } else if (!group_fits(n, ke - ks, ve - vs, total, hash_w)) {
    const uint64_t need = e2_need(total, hash_w);
    flags = need <= kImgMedium ? kPlanMedium : need <= kImgBig ? kPlanBig : kPlanHuge;
  }
  const BlockPlan pl{(uint32_t)recs, bin_len, hash_w, step | (flags << 8)};
  const uint64_t size = (bad ? 0 : total) | ((flags & (kPlanMedium | kPlanBig | kPlanHuge)) ? kListedOne : 0);
  P.plans[b] = pl;
  if (kFused) {
    fplan[tid] = pl;
    fsize[tid] = size;
    // (a listed block's status until its list kernel writes it: stays if the run's
    // output offset never arrives, see run_lookback)
    if (size & ~kOffMask) P.status[b] = ST_INCOMPLETE;
  } else {
    P.sizes[b] = size;
  }
  P.kspan[b] = ks;
  P.vspan[b] = vs;
  if (b + 1 == P.n_blocks) {
    P.kspan[b + 1] = ke;
    P.vspan[b + 1] = ve;
  }
}

template <bool kBkt, int kOW>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void encode_plan_wave_kernel(EncodeParams P) {
  __shared__ PlanWaveLds S;
  const uint32_t b0 = blockIdx.x * P.plan_bpw;
  plan_wave_run<kBkt, kOW, false>(P, b0, min(P.plan_bpw, P.n_blocks - b0), S, nullptr, nullptr);
}

// ------------------------------------------------ E2: group write kernel
// One 4-wave workgroup owns kGRun consecutive blocks and writes them in
// GROUPS: the longest run of consecutive group-class blocks whose items,
// key bytes, value bytes, encoded bytes and hash-index buckets fit the LDS
// budget (one 4 KiB data block is ~1/4 of a group; a 16 KiB one fills it).
// Consecutive blocks' items are contiguous in the arenas and their encoded
// bytes are contiguous in the output, so per group:
//   DMA    key and value spans HBM -> LDS stage (global_load_lds, 1 KiB per
//          wave instruction); thread t loads item t's offsets, seqno, type
//   shape  thread = item: shared prefix with its restart head (from the
//          stage), record length, workgroup scan -> record offset in block
//   write  thread = item: its record (header bytes, key suffix, value LEB +
//          bytes) into the LDS image of the group's output span, binary
//          index entry, hash-index vote; the next group's DMA is issued
//   tails  wave per block: marker, hash-index bytes, trailer
//   hash   the 16 DPP rows of the workgroup split every block's payload
//          into 1 KiB units (XXH3 per-KiB contributions, then one short
//          serial scramble chain per block)
//   header wave 0, lane per block: header fields + 29-byte checksum
//   out    16 B/lane copy of the group's span: the header-free pieces by three waves
//          while the fourth runs the chains, then the header pieces
// Blocks that do not fit are written by the list / HBM kernels.
struct GBlk {
  uint32_t it0, n;         // first item (group-relative), items
  uint32_t img, plen;      // header position in the image, payload length
  uint32_t recs, bin_len;  // record bytes, restart heads
  uint32_t step, hash_w;   // binary-index step, hash-index buckets
  uint32_t hash_base, u0;  // first vote pair, first hash unit
  uint32_t nbk, spare;     // full KiB units of the payload
};
static_assert(sizeof(GBlk) == 48, "GBlk");

struct GroupLds {
  uint8_t keys[kGKeys + kGSlack];
  uint8_t vals[kGVals + kGSlack];
  uint8_t img[kGImg + kGSlack];
  uint32_t uni[kGUnion / 4];
  GBlk blk[2][kGBlocks];  // this group's block table and the next one's (built under the chain)
  LongSecret secret;
};
// (the fused kernel's run-level plan keeps its LDS over vals + img, and its per-block
// outputs in uni, before the first group's DMA)
static_assert(offsetof(GroupLds, uni) - offsetof(GroupLds, vals) >= sizeof(PlanWaveLds), "plan LDS over the stage");
static_assert(offsetof(GroupLds, vals) % 16 == 0, "plan LDS alignment");
static_assert(kGRunFused * (sizeof(BlockPlan) + 8) + 16 <= kGUnion, "fused plan outputs in uni");


// n bytes src[s ..) (LDS) -> dst[d ..) (LDS): byte stores for the dst bytes
// that share a dword with a neighbour record, aligned dword stores inside
// (each from two source dwords and v_alignbyte); reads up to 8 bytes past.
// Lane `rot` starts its dword loop at a lane-dependent point of the span and
// wraps: records with a power-of-two source stride (64 B values: every lane
// of a 32-lane group on 2 banks) then read and write conflict-free.
__device__ __forceinline__ void lds_copy(uint8_t* dst, uint32_t d, const uint8_t* src, uint32_t s, uint32_t n,
                                         uint32_t rot) {
  if (!n) return;
  // (every read of a step is issued before its writes: one LDS round trip per step)
  const uint32_t h = min(n, (4u - (d & 3u)) & 3u);
  uint32_t hb[3];
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k)
    if (k < h) hb[k] = src[s + k];
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k)
    if (k < h) dst[d + k] = (uint8_t)hb[k];
  if (n == h) return;
  const uint32_t d1 = d + h, e = d + n, body = ((e & ~3u) - d1) >> 2;
  const uint32_t sp = s + h, sh = sp & 3u;
  const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src + (sp & ~3u));
  uint32_t* d32 = reinterpret_cast<uint32_t*>(dst + d1);
  // 32 start points: a ds_read_b32 wave access is two groups of 32 lanes, so
  // lanes with a 64-B source stride (16 dwords: two per bank) all differ.
  uint32_t q = ((rot & 31u) * body) >> 5;  // 0 <= q < body
  constexpr uint32_t U = 4;  // dwords per step (all reads before the writes)
  // Each source dword is read once: destination dword p is
  // alignbyte(src[p + 1], src[p]) and src[p] is the previous step's src[p + 1],
  // except after the wrap to p = 0, which takes w0 = src[0].
  const uint32_t w0 = body ? s32[0] : 0;
  uint32_t carry = body ? s32[q] : 0;
  for (uint32_t j0 = 0; j0 < body; j0 += U) {
    uint32_t hi[U], at[U];
#pragma unroll
    for (uint32_t t = 0; t < U; ++t) {
      uint32_t p = q + t;
      p = p >= body ? p - body : p;
      at[t] = p;
      if (j0 + t < body) hi[t] = s32[p + 1];
    }
#pragma unroll
    for (uint32_t t = 0; t < U; ++t) {
      if (j0 + t < body) {
        const uint32_t lo = t == 0 ? carry : (at[t] == 0 ? w0 : hi[t - 1]);
        d32[at[t]] = alignbyte(hi[t], lo, sh);
      }
    }
    q += U;
    q = q >= body ? q - body : q;
    carry = q == 0 ? w0 : hi[U - 1];
  }
  const uint32_t t0 = d1 + 4 * body;  // 0..3 tail bytes
  uint32_t tb[3];
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k)
    if (t0 + k < e) tb[k] = src[s + (t0 + k - d)];
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k)
    if (t0 + k < e) dst[t0 + k] = (uint8_t)tb[k];
}

__device__ __forceinline__ uint32_t lds_put_leb(uint8_t* dst, uint32_t pos, uint64_t v) {
  while (v >= 0x80) {
    dst[pos++] = (uint8_t)(v | 0x80);
    v >>= 7;
  }
  dst[pos++] = (uint8_t)v;
  return pos;
}

__device__ __forceinline__ void group_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// The group kernel's barrier: a release fence on LDS counts in-flight LDS-DMA
// as LDS stores and waits for it and for every other outstanding load
// (vmcnt(0)), which would expose the next group's stage DMA and item loads at
// the first barrier after they are issued.  Only this wave's own LDS
// operations are completed here (lgkmcnt(0)); the asm's memory clobber keeps
// the compiler from moving memory operations across it.  The stage and the
// prefetched item fields are waited for explicitly (vmcnt(0)) before the
// copy-out, and the next iteration's first barrier orders every wave's wait
// before any read of the stage.
__device__ __forceinline__ void group_barrier_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

#ifdef LSM_DIAG
// Diagnostic per-phase cycle totals of wave 0 of every group workgroup
// (lsm_block_params.reserved bit 0x80; read by lsm_diag_encode_phases).
#define ENC_PHASE(i)                                 \
  if (P.diag & 0x80) {                              \
    const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    ph_acc[i] += (uint32_t)(t_ - t_last);            \
    t_last = t_;                                     \
  }
#else
#define ENC_PHASE(i)
#endif

// kIndex: index blocks (restart interval 1, handle fields); kHash: the batch
// has hash indexes (hash ratio > 0).  Both are batch-wide, so the paths a
// batch never takes are compiled out (their registers would spill the
// common path: every scratch reload waits for all outstanding loads).
// ---------------------------------------- E1p: the plan of huge-block batches
// Blocks of ~4 Ki items and more on average (the writer's 1-4 MiB data blocks,
// writer/mod.rs:193-198) leave encode_plan_kernel one workgroup per one to four
// blocks, walking 512-item chunks one after another (60 workgroups for 60 blocks
// of 4 MiB: 0.21 ms for 240 x 1 MiB).  E1p computes the same outputs item-parallel:
//   lengths  thread per item: fields, shared prefix with its restart head
//            (encoder.rs:140-143), record length -> erec (for now), shared
//            length -> hbucket (unused by these batches' E2), per-block exact
//            record totals and bad flags (wave-segmented sums: a block's total,
//            or the parts at a wave's two ends)
//   scan     the device scan over every item's record length, in place (low
//            32 bits: a block's offsets are differences of two prefixes)
//   blocks   wave per block: its total from the wave parts, the plan as
//            encode_plan_kernel's epilogue
//   offsets  thread per item: erec = prefix - its block's first prefix (the
//            packed word for blocks of <= kGItems items); huge blocks keep the
//            prefix (their writers subtract pfirst)
// A non-monotone item_start array rejects every block (the one-workgroup
// plan rejects the run of blocks its workgroup holds).
__device__ __forceinline__ uint32_t block_of_item(const EncodeParams& P, uint32_t i) {
  uint32_t lo = 0, hi = P.n_blocks;  // last b < n_blocks with start[b] <= i
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (clamped_start(P, mid) <= i) lo = mid;
    else hi = mid;
  }
  return lo;
}

constexpr uint64_t kE1pBad = 1ULL << 63;
constexpr uint32_t kE1pMaxBpw = 4;  // E1p for batches of >= 4 Ki items per block on average
// Sum of two (record bytes | bad flag) words.
__device__ __forceinline__ uint64_t e1p_add(uint64_t a, uint64_t b) {
  return ((a | b) & kE1pBad) | ((a + b) & ~kE1pBad);
}

__device__ __forceinline__ uint64_t shfl_down64(uint64_t v, int o) {
  return (uint64_t)(uint32_t)__shfl_down((int)(uint32_t)v, o) |
         ((uint64_t)(uint32_t)__shfl_down((int)(uint32_t)(v >> 32), o) << 32);
}

// Items per thread in the item-parallel E1p kernels (strided by 256: each pass
// of a workgroup is 256 consecutive items); the four items' loads are issued
// together, and a workgroup's block search serves 1024 items.
constexpr uint32_t kE1pPer = 4;
constexpr uint32_t kE1pLenPer = 1;  // (the lengths kernel: 4 items took 136 VGPRs, 2 ran as 1)

// The block holding item `first` (the workgroup's first item), by a 256-way
// search of the starts (every thread one sample per round: one round for
// batches of <= 256 blocks; a thread-0 binary search was eight dependent loads
// before any item load of the workgroup).  Every thread calls it (a barrier).
__device__ __forceinline__ uint32_t wg_first_block(const EncodeParams& P, uint32_t first) {
  const uint32_t i_end = clamped_start(P, P.n_blocks);
  uint32_t lo = 0, hi = P.n_blocks;  // last b in [lo, hi) with start[b] <= first
  if (first >= i_end) hi = 1;       // (no item of the batch here: block 0, unused)
  while (hi - lo > 1) {             // (uniform)
    const uint32_t st = (hi - lo + 255) / 256;
    const uint32_t x = lo + threadIdx.x * st;
    const uint32_t c = (uint32_t)__syncthreads_count(x < hi && clamped_start(P, x) <= first);
    const uint32_t nlo = lo + (c ? c - 1 : 0) * st;  // (c = 0 only for a non-monotone array: rejected anyway)
    hi = min(hi, nlo + st);
    lo = nlo;
  }
  return lo;
}

// This thread's kE1pPer items (base + 256 j + tid): each one's block and range,
// walking forward from the workgroup's first block (blocks of >= 4 Ki items on
// average: a step or two at most).
template <uint32_t K>
struct E1pItems {
  uint32_t i[K], b[K], s[K], e[K];
  bool in[K];
};
template <uint32_t K>
__device__ __forceinline__ E1pItems<K> e1p_items(const EncodeParams& P) {
  E1pItems<K> t;
  const uint32_t i_begin = clamped_start(P, 0), i_end = clamped_start(P, P.n_blocks);
  const uint32_t base = blockIdx.x * (256 * K);
  uint32_t b = wg_first_block(P, max(base, i_begin));
  uint32_t bs = clamped_start(P, b), be = clamped_start(P, b + 1);
#pragma unroll
  for (uint32_t j = 0; j < K; ++j) {
    const uint32_t i = base + 256 * j + threadIdx.x;
    const bool in = i >= i_begin && i < i_end && (uint64_t)i < P.it.n_items;
    while (in && b + 1 < P.n_blocks && be <= i) {
      ++b;
      bs = be;
      be = clamped_start(P, b + 1);
    }
    t.i[j] = i;
    t.b[j] = b;
    t.s[j] = bs;
    t.e[j] = be;
    t.in[j] = in;
  }
  return t;
}

// The huge-block pool header's collected-block count (EncHugeHdr::count), as a u32 index.
constexpr uint32_t kEncHugeCountWord = 2;

template <int kOW>
__global__ __launch_bounds__(256) void encode_e1p_lengths_kernel(EncodeParams P) {
  if (blockIdx.x == 0) {  // the starts' monotonicity over every block, the flag written whole (no prior clear)
    int bad = 0;
    for (uint32_t x = threadIdx.x; x < P.n_blocks; x += 256)
      bad |= clamped_start(P, x + 1) < clamped_start(P, x) ? 1 : 0;
    bad = __syncthreads_or(bad);
    if (threadIdx.x == 0) {
      P.e1p_flag[0] = bad ? 1u : 0u;
      if (P.huge_pool) reinterpret_cast<uint32_t*>(P.huge_pool)[kEncHugeCountWord] = 0;  // (the size scan counts into it)
    }
  }
  const E1pItems<kE1pLenPer> T = e1p_items<kE1pLenPer>(P);
  const uint32_t ri = P.ri, lane = threadIdx.x & 63;
  bool live[kE1pLenPer], head[kE1pLenPer];
  RawItemT<kOW> r[kE1pLenPer];
  uint64_t hko[kE1pLenPer], hko1[kE1pLenPer];
#pragma unroll
  for (uint32_t j = 0; j < kE1pLenPer; ++j) {  // every item's loads first
    const uint32_t i = T.i[j];
    live[j] = T.in[j] && T.s[j] <= i && i < T.e[j];  // (not, for a non-monotone array: every block is rejected)
    head[j] = (i - T.s[j]) % ri == 0;
    hko[j] = hko1[j] = 0;
    if (live[j]) {
      r[j] = load_raw<false, kOW>(P, i);
      if (!head[j]) {
        const uint64_t h = (uint64_t)i - (i - T.s[j]) % ri;
        hko[j] = koff<kOW>(P, h);
        hko1[j] = koff<kOW>(P, h + 1);
      }
    }
  }
  ItemMeta m[kE1pLenPer];
  bool bad[kE1pLenPer];
  Win16 wa[kE1pLenPer], wb[kE1pLenPer];
#pragma unroll
  for (uint32_t j = 0; j < kE1pLenPer; ++j) {  // then the key windows of the shared prefixes
    bad[j] = false;
    if (live[j]) {
      m[j] = cook_item<false>(r[j], bad[j]);
      if (!head[j]) {
        wa[j] = gwin16(P.it.keys + hko[j]);
        wb[j] = gwin16(P.it.keys + m[j].ko);
      }
    }
  }
#pragma unroll
  for (uint32_t j = 0; j < kE1pLenPer; ++j) {
    const uint32_t i = T.i[j];
    uint64_t rec = 0;
    if (live[j]) {
      if (!head[j]) {
        const uint32_t n = min((uint32_t)min(hko1[j] - hko[j], (uint64_t)0xFFFF), m[j].klen);
        const uint64_t x0 = wa[j].lo ^ wb[j].lo, x1 = wa[j].hi ^ wb[j].hi;
        uint32_t sh;
        if (x0) sh = min(n, (uint32_t)(__builtin_ctzll(x0) >> 3));
        else if (x1) sh = min(n, 8 + (uint32_t)(__builtin_ctzll(x1) >> 3));
        else sh = n <= 16 ? n : lcp_tail(P.it.keys, hko[j], m[j].ko, n);
        m[j].sh = sh;
        P.hbucket[i] = (uint16_t)min(sh, 0xFFFFu);
      }
      rec = item_record_len(P, m[j], head[j]);
    }
    if ((uint64_t)i < P.it.n_items) P.erec[i] = (uint32_t)min(rec, (uint64_t)0xFFFFFFFFu);
    // per-block exact totals without same-address atomics (a 4-MiB block's ~800
    // waves would serialise on one word): lanes of one block summed first (blocks
    // are runs of lanes); a block inside this wave stores its total, one that began
    // in an earlier wave its part as this wave's head, one that goes on past this
    // wave its part as this wave's tail (encode_e1p_blocks_kernel adds them up)
    const uint32_t b = T.b[j], s = T.s[j], e = T.e[j];
    const uint32_t bb = live[j] ? b : 0xFFFFFFFFu;
    uint64_t sum = rec | (bad[j] ? kE1pBad : 0);
    for (int o = 1; o < 64; o <<= 1) {  // segmented wave reduction: run heads end with their run's total
      const uint64_t v = shfl_down64(sum, o);
      const uint32_t bo = (uint32_t)__shfl_down((int)bb, o);
      if ((int)lane + o < 64 && bo == bb) sum = e1p_add(sum, v);
    }
    const uint32_t bprev = (uint32_t)__shfl_up((int)bb, 1);
    if (live[j] && (lane == 0 || bprev != bb)) {
      const uint32_t w0 = i - lane;
      if (s >= w0 && e - w0 <= 64) P.sizes[b] = sum;
      else if (s < w0) P.wpart[2 * (uint64_t)(w0 / 64)] = sum;
      else P.wpart[2 * (uint64_t)(w0 / 64) + 1] = sum;
    }
  }
}

// Scan output: each item's record prefix (low 32 bits) in place; the total in pfirst[n_blocks].
struct E1pOut {
  uint32_t* erec;
  uint32_t* total;
  uint64_t n;
  __device__ void operator()(uint64_t i, uint64_t prefix) const {
    if (i < n) erec[i] = (uint32_t)prefix;
    else *total = (uint32_t)prefix;
  }
};

__device__ __forceinline__ uint32_t e1p_prefix(const EncodeParams& P, uint32_t i) {
  return (uint64_t)i < P.it.n_items ? P.erec[i] : P.pfirst[P.n_blocks];
}

// Wave per block: its record total from the lengths kernel's per-wave parts,
// then the plan (encode_plan_kernel's epilogue) on lane 0.
__global__ __launch_bounds__(256) void encode_e1p_blocks_kernel(EncodeParams P) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t bq = ((uint64_t)blockIdx.x * 256 + threadIdx.x) / 64;
  if (bq >= P.n_blocks) return;  // (wave-uniform)
  const uint32_t b = (uint32_t)bq;
  const uint32_t ri = P.ri;
  const uint32_t s = clamped_start(P, b), e = clamped_start(P, b + 1);
  uint64_t acc = 0;
  if (e > s && !P.e1p_flag[0]) {
    const uint32_t ws = s / 64, we = (e - 1) / 64;
    if (ws == we) {
      acc = P.sizes[b];
    } else {
      uint64_t x = lane == 0 ? P.wpart[2 * (uint64_t)ws + 1] : 0;
      for (uint64_t w = (uint64_t)ws + 1 + lane; w <= we; w += 64) x = e1p_add(x, P.wpart[2 * w]);
      for (int o = 32; o; o >>= 1) x = e1p_add(x, shfl_xor64(x, o));
      acc = x;
    }
  }
  if (lane) return;
  bool bad = P.e1p_flag[0] || e <= s || (acc & kE1pBad) || start_past_items(P, b + 1);
  const uint32_t n = bad ? 0 : e - s;
  const uint64_t recs = bad ? 0 : acc & ~kE1pBad;
  const uint32_t p_s = bad ? 0 : e1p_prefix(P, s);
  P.pfirst[b] = p_s;
  const uint32_t bin_len = n ? (n + ri - 1) / ri : 0;
  const uint64_t last_head = n ? (uint32_t)(e1p_prefix(P, s + (bin_len - 1) * ri) - p_s) : 0;
  const uint32_t step = last_head <= 0xFFFF ? 2 : 4;
  const uint32_t buckets = bucket_count(n, P.ratio);
  const uint32_t hash_w = (buckets > 0 && bin_len <= kHashMaxPointers) ? buckets : 0;
  const uint64_t total = kHdrLen + recs + 1 + (uint64_t)bin_len * step + hash_w + kTrailerLen;
  if (recs > 0xFFFFFFF0ULL || total > 0xFFFFFF00ULL) bad = true;
  const uint64_t ks = koff(P, s), ke = koff(P, e);
  const uint64_t vs = voff(P, s), ve = voff(P, e);
  uint32_t flags = 0;
  if (bad) {
    flags = kPlanBad;
    P.status[b] = ST_BAD_ARG;
  } else if (!group_fits(n, ke - ks, ve - vs, total, hash_w)) {
    const uint64_t need = e2_need(total, hash_w);
    flags = need <= kImgMedium ? kPlanMedium : need <= kImgBig ? kPlanBig : kPlanHuge;
  }
  P.plans[b] = BlockPlan{(uint32_t)recs, bin_len, hash_w, step | (flags << 8)};
  P.sizes[b] = (bad ? 0 : total) | ((flags & (kPlanMedium | kPlanBig | kPlanHuge)) ? kListedOne : 0);
  P.kspan[b] = ks;
  P.vspan[b] = vs;
  if (b + 1 == P.n_blocks) {
    P.kspan[b + 1] = ke;
    P.vspan[b + 1] = ve;
  }
}

__global__ __launch_bounds__(256) void encode_e1p_offsets_kernel(EncodeParams P) {
  const E1pItems<kE1pPer> T = e1p_items<kE1pPer>(P);
  if (P.e1p_flag[0]) return;
  const uint32_t ri = P.ri;
  // (huge blocks keep the record prefix in erec: their writers subtract the block's first
  // prefix themselves, so their items, nearly all of such a batch, cost only the flag load here)
  uint32_t fl[kE1pPer], er[kE1pPer], pf[kE1pPer], hb[kE1pPer];
  bool cv[kE1pPer];
#pragma unroll
  for (uint32_t j = 0; j < kE1pPer; ++j) fl[j] = T.in[j] ? gload_pod(P.plans, T.b[j]).step_flags : 0;
#pragma unroll
  for (uint32_t j = 0; j < kE1pPer; ++j) {  // every converted item's loads first
    er[j] = pf[j] = hb[j] = 0;
    cv[j] = T.in[j] && !((fl[j] >> 8) & kPlanBad) && (fl[j] >> 8) != kPlanHuge;
    if (cv[j]) {
      er[j] = gload(P.erec, T.i[j]);
      pf[j] = gload(P.pfirst, T.b[j]);
      hb[j] = gload(P.hbucket, T.i[j]);
    }
  }
#pragma unroll
  for (uint32_t j = 0; j < kE1pPer; ++j) {
    if (!cv[j]) continue;
    const uint32_t n = T.e[j] - T.s[j], roff = er[j] - pf[j], jj = T.i[j] - T.s[j];
    const bool head = jj % ri == 0;
    const uint32_t x = head ? jj / ri : hb[j];
    P.erec[T.i[j]] = n > kGItems ? roff : min(roff, 0x7FFFu) | (head ? kErecHead : 0u) | (min(x, 0xFFFFu) << 16);
  }
}

// The buckets of the keys E1 left (more than 16 bytes): a wave per block,
// grid-stride; exits at once when E1 left none.
__global__ __launch_bounds__(256) void encode_bucket_fixup_kernel(EncodeParams P) {
  if (!P.hb_fix[0]) return;
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const uint32_t w0 = (blockIdx.x * blockDim.x + threadIdx.x) / kWave, nw = gridDim.x * blockDim.x / kWave;
  for (uint32_t b = w0; b < P.n_blocks; b += nw) {
    // blocks E1 rejected (non-monotone or out-of-range starts, over-long keys,
    // bad value types) are skipped by E2: their hbucket entries may be stale
    if ((P.plans[b].step_flags >> 8) & kPlanBad) continue;
    const uint32_t s = P.starts[b], e = P.starts[b + 1];  // (E1 checked s < e <= n_items)
    const uint32_t n = e - s, buckets = bucket_count(n, P.ratio);
    const uint32_t hw = (buckets > 0 && (n + P.ri - 1) / P.ri <= kHashMaxPointers) ? buckets : 0;
    if (!hw || hw >= kNeedHash) continue;
    for (uint32_t i = s + lane; i < e; i += kWave) {
      if (P.hbucket[i] != kNeedHash) continue;
      const uint64_t ko = koff(P, i);
      // (E1 checked every key of a good block: <= 0xFFFF bytes; the cap is the same as E1's)
      const uint32_t klen = (uint32_t)min(koff(P, i + 1) - ko, (uint64_t)0xFFFF);
      const uint64_t hv = xxh3_64_any(klen, BaseReader8{P.it.keys + ko, 0}, BaseReader64{P.it.keys + ko, 0});
      P.hbucket[i] = (uint16_t)(hv % hw);
    }
  }
}

// ---- the fused plan's run offsets: a decoupled look-back over the runs (one word per
// run in P.sizes, cleared before the launch): bits 62-63 the state (1: this run's own
// bytes, 2: the inclusive prefix through this run), bit 61 poison, bits 0-60 the value
// (output bytes in bits 0-39, listed blocks above, as P.sizes' words).  A run publishes
// its own total as soon as its plan is done, before it looks back, and looks back only
// at lower runs, which were dispatched before it: every wait ends.  The wait is also
// bounded in time (100 ms without progress): a run that gives up publishes poison, and
// its blocks and every later run's report LSM_INCOMPLETE instead of bytes at a wrong
// offset.
constexpr uint64_t kLbAgg = 1ULL << 62, kLbIncl = 2ULL << 62, kLbPoison = 1ULL << 61, kLbVal = kLbPoison - 1;
constexpr uint64_t kLookbackTicks = 10000000;  // s_memrealtime runs at 100 MHz
// diagnostic builds: lsm_block_params.reserved bit 0x20 makes every run but the first give up
// at once (tests/test_gpu_encode_fused.py checks the poison path end to end)
constexpr uint32_t kDiagLookbackGiveUp = 0x20;

__device__ __forceinline__ uint64_t lb_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One wave: publishes `agg` for `run`, returns the sum of the runs before it.
__device__ __noinline__ uint64_t run_lookback(uint64_t* lb, uint32_t run, uint64_t agg, uint32_t diag, bool& poisoned) {
  const int lane = threadIdx.x & (kWave - 1);
  if (lane == 0) lb_store(lb + run, (run == 0 ? kLbIncl : kLbAgg) | agg);
  uint64_t excl = 0;
  bool poison = false;
  if (run != 0) {
    int64_t top = (int64_t)run - 1;  // lane l looks at run top - l
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      const int64_t idx = top - lane;
      const uint64_t v = idx >= 0 ? lb_load(lb + idx) : kLbIncl;  // (before run 0: an inclusive 0)
      const uint64_t incl_m = __ballot((v >> 62) == 2), ready_m = __ballot((v >> 62) != 0);
      const uint32_t stop = incl_m ? (uint32_t)__builtin_ctzll(incl_m) : 64u;  // the nearest inclusive prefix
      const uint64_t need = stop >= 63 ? ~0ULL : (2ULL << stop) - 1;
      if ((ready_m & need) == need && !(kDiagBuild && (diag & kDiagLookbackGiveUp))) {
        const bool mine = (uint32_t)lane <= stop;
        poison = poison || __ballot(mine && (v & kLbPoison)) != 0;
        excl += wave_bcast_u64(wave_incl_scan_u64(mine ? (v & kLbVal) : 0), kWave - 1);
        if (stop < 64) break;
        top -= 64;
        t0 = __builtin_amdgcn_s_memrealtime();
        continue;
      }
      if (__builtin_amdgcn_s_memrealtime() - t0 > kLookbackTicks || (kDiagBuild && (diag & kDiagLookbackGiveUp))) {
        poison = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (lane == 0) lb_store(lb + run, kLbIncl | (poison ? kLbPoison : 0) | ((excl + agg) & kLbVal));
  }
  poisoned = poison;
  return excl;
}

template <bool kIndex, bool kHash, bool kPlanBkt, int kOW, bool kFused = false>
__global__ __launch_bounds__(kGThreads) __attribute__((amdgpu_waves_per_eu(4))) void encode_group_kernel(EncodeParams P) {
  static_assert(!kFused || (!kIndex && !kHash), "the fused plan is for data blocks without a hash index");
  __shared__ GroupLds L;
  typedef __attribute__((address_space(3))) void lds_void_t;
  typedef const __attribute__((address_space(1))) void gbl_void_t;
  const uint32_t tid = threadIdx.x;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int lane = tid & (kWave - 1);
  constexpr uint32_t kRun = kFused ? kGRunFused : kGRun;
  const uint32_t b_begin = blockIdx.x * kRun;
  const uint32_t b_end = min(b_begin + kRun, P.n_blocks);
  const uint32_t ri = kIndex ? 1 : P.ri;
  constexpr bool index = kIndex;
  if (tid < sizeof(LongSecret) / 8)
    reinterpret_cast<uint64_t*>(&L.secret)[tid] = reinterpret_cast<const uint64_t*>(&kLongSecret)[tid];
  // the run's blocks, lane l = block b_begin + l (every wave holds the same registers)
  const uint32_t rb = b_begin + lane;
  const bool in_run = rb <= b_end;
  const uint32_t r_start = in_run ? P.starts[rb] : 0;
  uint64_t r_off, r_ks, r_vs;
  BlockPlan r_plan;
  bool run_ok = true;
  if (kFused) {
    // the plan pass's code on this run's blocks (its LDS over the stage, before the first
    // DMA), then the run's output offset by the look-back: no plan launch, no size scan,
    // and the item fields and keys this loop reads again are the ones the plan just read
    BlockPlan* const fplan = reinterpret_cast<BlockPlan*>(L.uni);               // [kRun]
    uint64_t* const fsize = reinterpret_cast<uint64_t*>(L.uni) + 2 * kRun;      // [kRun]
    uint64_t* const fbase = fsize + kRun;                                       // prefix, poison
    plan_wave_run<false, kOW, true>(P, b_begin, b_end - b_begin, *reinterpret_cast<PlanWaveLds*>(L.vals), fplan,
                                    fsize);
    __syncthreads();
    r_plan = rb < b_end ? fplan[lane] : BlockPlan{0, 0, 0, 0};
    const uint64_t sz = rb < b_end ? fsize[lane] : 0;
    const uint64_t incl = wave_incl_scan_u64(sz);
    if (wave == 0) {
      bool poisoned;
      const uint64_t base = run_lookback(P.sizes, blockIdx.x, wave_bcast_u64(incl, kWave - 1), P.diag, poisoned);
      if (lane == 0) {
        fbase[0] = base;
        fbase[1] = poisoned ? 1 : 0;
      }
    }
    __syncthreads();
    const uint64_t ex = fbase[0] + incl - sz;
    run_ok = fbase[1] == 0;
    r_off = in_run ? (ex & kOffMask) : 0;
    if (wave == 0 && rb < b_end) {
      P.block_off[rb] = r_off;
      if (!run_ok) P.status[rb] = ST_INCOMPLETE;
      else if (sz & ~kOffMask) P.lists[ex >> 40] = rb;
    }
    if (wave == 0 && rb == b_end && b_end == P.n_blocks) {  // the last run: the total and the list length
      P.block_off[rb] = r_off;
      P.list_count[0] = run_ok ? (uint32_t)(ex >> 40) : 0u;
    }
    const uint32_t cs = in_run ? clamped_start(P, rb) : 0;
    r_ks = in_run ? koff<kOW>(P, cs) : 0;
    r_vs = in_run ? voff<kOW>(P, cs) : 0;
    __syncthreads();  // (L.uni is the group loop's from here)
  } else {
    r_off = in_run ? P.block_off[rb] : 0;
    r_ks = in_run ? P.kspan[rb] : 0;
    r_vs = in_run ? P.vspan[rb] : 0;
    r_plan = (in_run && rb < b_end) ? P.plans[rb] : BlockPlan{0, 0, 0, 0};
  }
  const uint32_t r_hash = r_plan.hash_w;
  const uint32_t r_hpre = wave_incl_scan_u32(r_hash) - r_hash;  // exclusive prefix over the run
  // payload hash units (1 KiB, long path only) per block, exclusive prefix over the run
  uint32_t r_upre;
  {
    const uint64_t nx = wave_shfl_u64(r_off, min(lane + 1, 63));
    const uint32_t plen = (rb < b_end) ? (uint32_t)(nx - r_off) - kHdrLen : 0;
    const uint32_t units = plen > 240 ? (plen - 1) / 1024 + 1 : 0;
    r_upre = wave_incl_scan_u32(units) - units;
  }
  auto lane_u32 = [&](uint32_t v, uint32_t l) { return (uint32_t)__shfl((int)v, (int)min(l, 63u)); };
  auto lane_u64 = [&](uint64_t v, uint32_t l) { return wave_shfl_u64(v, (int)min(l, 63u)); };
  // the same for a wave-uniform lane index: v_readlane into a scalar register
  auto rl32 = [&](uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)min(l, 63u)); };
  auto rl64 = [&](uint64_t v, uint32_t l) {
    const int q = (int)min(l, 63u);
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, q) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), q) << 32);
  };
  struct Grp {
    uint32_t b, k;
  };
  // the longest group from block b (k = 0: block b is listed / rejected / over capacity)
  auto form = [&](uint32_t b) -> Grp {
    const uint32_t r0 = b - b_begin, rj = r0 + lane;
    const uint32_t s0 = rl32(r_start, r0), s1 = lane_u32(r_start, rj + 1);
    const uint64_t o0 = rl64(r_off, r0), o1 = lane_u64(r_off, rj + 1);
    const uint64_t k0 = rl64(r_ks, r0), k1 = lane_u64(r_ks, rj + 1);
    const uint64_t v0 = rl64(r_vs, r0), v1 = lane_u64(r_vs, rj + 1);
    const uint32_t flags = lane_u32(r_plan.step_flags, rj) >> 8;
    const uint32_t hsum = lane_u32(r_hpre, rj + 1) - rl32(r_hpre, r0);
    const bool ok = b + lane < b_end && lane < (int)kGBlocks && flags == 0 && o1 <= P.out_cap &&
                    group_fits(s1 - s0, k1 - (k0 & ~15ULL), v1 - (v0 & ~15ULL), o1 - (o0 & ~15ULL), hsum);
    return Grp{b, (uint32_t)__builtin_ctzll(~__ballot(ok))};
  };
  // the run's group-class blocks (listed / rejected ones are passed over at once)
  const uint64_t gmask = __ballot(rb < b_end && (r_plan.step_flags >> 8) == 0);
  auto next_group = [&](uint32_t b) -> Grp {
    for (;;) {
      if (b >= b_end) return Grp{b, 0};
      const Grp g = form(b);
      if (g.k) return g;
      const uint64_t rest = gmask >> (b - b_begin);
      if (rest & 1) {
        if (lane == 0) P.status[b] = ST_OVERFLOW;  // group class, but past out_cap
        ++b;
      } else {
        b = rest ? b + (uint32_t)__builtin_ctzll(rest) : b_end;
      }
    }
  };
  auto issue_dma = [&](const Grp& g) {
    const uint32_t r0 = g.b - b_begin;
    const uint64_t ka = rl64(r_ks, r0) & ~15ULL, kb = rl64(r_ks, r0 + g.k);
    const uint64_t va = rl64(r_vs, r0) & ~15ULL, vb = rl64(r_vs, r0 + g.k);
    const uint32_t kc = (uint32_t)((kb - ka + 15) >> 4), vc = index ? 0 : (uint32_t)((vb - va + 15) >> 4);
    const uint8_t* ks = P.it.keys + ka + 16 * lane;
    for (uint32_t i = wave; i * kWave < kc; i += kGWaves)
      if (i * kWave + lane < kc)
        __builtin_amdgcn_global_load_lds((gbl_void_t*)(ks + 1024 * i), (lds_void_t*)(L.keys + 1024 * i), 16, 0, 0);
    const uint8_t* vs = P.it.vals + va + 16 * lane;
    for (uint32_t i = wave; i * kWave < vc; i += kGWaves)
      if (i * kWave + lane < vc)
        __builtin_amdgcn_global_load_lds((gbl_void_t*)(vs + 1024 * i), (lds_void_t*)(L.vals + 1024 * i), 16, 0, 0);
  };
  uint32_t* hlo = L.uni;                           // [kGHash] vote min
  uint32_t* hhi = hlo + kGHash;                    // [kGHash] vote max
  uint64_t* contrib = reinterpret_cast<uint64_t*>(L.uni);  // [kGUnits][4][2] (after the records)

  // item t's raw fields of group g: plain loads, no arithmetic and no branch
  // (threads past the group's items load its last item), so nothing waits
  // for them until the next iteration cooks them (the plan pass has vetted
  // every group-class item: no `bad` checks here)
  // Groups of few items (16 KiB blocks of long values: 56 items) give each
  // item 2 or 4 threads (tpi = 1 << tsh), which split its value copy; thread t
  // serves item t >> tsh, part t & (tpi - 1).
  auto tpi_shift = [&](uint32_t n) -> uint32_t { return n <= kGThreads / 4 ? 2u : n <= kGThreads / 2 ? 1u : 0u; };
  auto load_items = [&](const Grp& g, RawItemT<kOW, kIndex>& r) {
    const uint32_t r0 = g.b - b_begin;
    const uint32_t i0 = rl32(r_start, r0), n = rl32(r_start, r0 + g.k) - i0;
    const uint64_t i = (uint64_t)i0 + min(tid >> tpi_shift(n), n - 1);
    r = load_raw<kIndex, kOW>(P, i);
    r.e = P.erec[i];
    if (kPlanBkt) r.hb = P.hbucket[i];
  };
  auto cook = [&](const RawItemT<kOW, kIndex>& r) {
    bool bad = false;  // (vetted by the plan pass)
    return cook_item<kIndex>(r, bad);
  };

  // group g's block table (lane j = block j; one wave, every lane active for the shuffles)
  auto build_table = [&](const Grp& g, GBlk* tb) {
    const uint32_t gr0 = g.b - b_begin, gk = g.k;
    const uint32_t gi0 = rl32(r_start, gr0);
    const uint64_t gob = rl64(r_off, gr0);
    const uint32_t gpad = (uint32_t)(((uint64_t)(uintptr_t)P.out + gob) & 15);
    const uint32_t rj = gr0 + lane;
    const uint32_t st = lane_u32(r_start, rj), st1 = lane_u32(r_start, rj + 1);
    const uint64_t of = lane_u64(r_off, rj), of1 = lane_u64(r_off, rj + 1);
    const uint32_t recs = lane_u32(r_plan.recs, rj), bin_len = lane_u32(r_plan.bin_len, rj);
    const uint32_t sf = lane_u32(r_plan.step_flags, rj), hw = lane_u32(r_plan.hash_w, rj);
    const uint32_t hb = lane_u32(r_hpre, rj) - rl32(r_hpre, gr0);
    const bool in = (uint32_t)lane < gk;
    const uint32_t plen = in ? (uint32_t)(of1 - of) - kHdrLen : 0;
    const uint32_t nbk = plen > 240 ? (plen - 1) / 1024 : 0;
    const uint32_t units = plen > 240 ? nbk + 1 : 0;
    const uint32_t u0 = wave_incl_scan_u32(units) - units;
    if (in) {
      GBlk B;
      B.it0 = st - gi0;
      B.n = st1 - st;
      B.img = (uint32_t)(of - gob) + gpad;
      B.plen = plen;
      B.recs = recs;
      B.bin_len = bin_len;
      B.step = sf & 0xFF;
      B.hash_w = hw;
      B.hash_base = hb;
      B.u0 = u0;
      B.nbk = nbk;
      B.spare = 0;
      tb[lane] = B;
    }
  };

  // Software pipeline: group G's stage DMA and item fields are issued one
  // group ahead and waited for (vmcnt(0)) just before the previous group's
  // copy-out, so no group waits on HBM latency after its stores.
#ifdef LSM_DIAG
  uint64_t t_last = __builtin_amdgcn_s_memtime();
  uint32_t ph_acc[12] = {};
  uint32_t ph_n = 0;
#endif
  Grp G = run_ok ? next_group(b_begin) : Grp{b_end, 0};
  RawItemT<kOW, kIndex> raw{};
  if (G.k) {
    issue_dma(G);
    load_items(G, raw);
    if (wave == 0) build_table(G, L.blk[0]);  // (later tables are built under the previous chain)
  }
  __builtin_amdgcn_s_waitcnt(0x0070);
  ENC_PHASE(11);
  uint32_t iter = 0;  // rotates the chain wave over the SIMDs
  while (G.k) {
    ENC_PHASE(0);
    const uint32_t r0 = G.b - b_begin, k = G.k;
    const uint32_t i0 = rl32(r_start, r0), n_items = rl32(r_start, r0 + k) - i0;
    const uint64_t kbase = rl64(r_ks, r0) & ~15ULL, vbase = rl64(r_vs, r0) & ~15ULL;
    const uint64_t obase = rl64(r_off, r0);
    const uint64_t dabs = (uint64_t)(uintptr_t)P.out + obase;
    const uint32_t pad = (uint32_t)(dabs & 15);
    const uint32_t tsh = tpi_shift(n_items), part = tid & ((1u << tsh) - 1), item = tid >> tsh;
    const bool live = item < n_items;
    // the next group's item fields: in flight under this whole group
    const Grp Gn = next_group(G.b + k);
    ItemMeta m = cook(raw);
    if (Gn.k) load_items(Gn, raw);
    ENC_PHASE(9);
    GBlk* const TB = L.blk[iter & 1];  // this group's block table (built one group ahead)
    // (shuffles only with every lane active: a bpermute from an inactive lane is undefined)
    const uint32_t hsum = rl32(r_hpre, r0 + k) - rl32(r_hpre, r0);
    for (uint32_t h = tid; h < hsum; h += kGThreads) {
      hlo[h] = 0xFFFFFFFFu;
      hhi[h] = 0;
    }
    group_barrier_lds();
    ENC_PHASE(1);
    // ---- item t: its block (record offset and shared prefix from E1)
    // (block starts from the run registers, v_readlane: no LDS round trip)
    uint32_t j = 0;
    for (uint32_t jb = 1; jb < k; ++jb) j += (rl32(r_start, r0 + jb) - i0 <= item) ? 1u : 0u;
    const bool head = (m.e & kErecHead) != 0;
    m.sh = head ? 0u : m.e >> 16;
    // ---- item t: its record into the image (one thread per item, or for
    // groups of few items tpi threads per item splitting the value copy)
    // Two writers on purpose: the split one (tsh > 0) also covers tsh = 0, but as
    // the only writer it measured 0.6 % slower on configs[1] and 0.5 % on
    // configs[3] (3.237 vs 3.218 ms, 3.131 vs 3.115 ms; profiles/r03_encode_experiments.txt).
    // A fix in one must be made in both.
    if (tsh == 0) {
    if (live && !(kDiagBuild && (P.diag & 9))) {
      const GBlk& B = TB[j];
      const uint32_t roff = m.e & 0x7FFFu;
      const uint32_t p0 = B.img + kHdrLen;
      uint32_t pos = p0 + roff;
      const uint32_t kst = (uint32_t)(m.ko - kbase);
      if (index) {
        L.img[pos++] = 0;
        pos = lds_put_leb(L.img, pos, m.vo);
        pos = lds_put_leb(L.img, pos, m.vl);
        pos = lds_put_leb(L.img, pos, m.seq);
        pos = lds_put_leb(L.img, pos, m.klen);
        lds_copy(L.img, pos, L.keys, kst, m.klen, lane);
      } else {
        L.img[pos++] = (uint8_t)m.vt;
        pos = lds_put_leb(L.img, pos, m.seq);
        const uint32_t from = head ? 0 : m.sh;
        if (!head) pos = lds_put_leb(L.img, pos, m.sh);
        pos = lds_put_leb(L.img, pos, m.klen - from);
        lds_copy(L.img, pos, L.keys, kst + from, m.klen - from, lane);
        pos += m.klen - from;
        if (!is_tombstone(m.vt)) {
          pos = lds_put_leb(L.img, pos, m.vl);
          lds_copy(L.img, pos, L.vals, (uint32_t)(m.vo - vbase), m.vl, lane);
        }
      }
      if (head) {
        const uint32_t bp = p0 + B.recs + 1 + (m.e >> 16) * B.step;
        for (uint32_t q = 0; q < B.step; ++q) L.img[bp + q] = (uint8_t)(roff >> (8 * q));
      }
      if (kHash && B.hash_w) {
        const uint32_t ridx = (tid - B.it0) / ri;
        const uint32_t hb =
            kPlanBkt ? m.hb
                     : (uint32_t)(xxh3_64_any(m.klen, BaseReader8{L.keys, kst}, BaseReader64{L.keys, kst}) % B.hash_w);
        const uint32_t bk = B.hash_base + hb;
        atomicMin(&hlo[bk], ridx);
        atomicMax(&hhi[bk], ridx);
      }
    }
    } else {
    if (live && !(kDiagBuild && (P.diag & 9))) {
      const GBlk& B = TB[j];
      const uint32_t roff = m.e & 0x7FFFu;
      const uint32_t p0 = B.img + kHdrLen;
      uint32_t pos = p0 + roff;
      const uint32_t kst = (uint32_t)(m.ko - kbase);
      if (index) {
        if (part == 0) {
          L.img[pos++] = 0;
          pos = lds_put_leb(L.img, pos, m.vo);
          pos = lds_put_leb(L.img, pos, m.vl);
          pos = lds_put_leb(L.img, pos, m.seq);
          pos = lds_put_leb(L.img, pos, m.klen);
          lds_copy(L.img, pos, L.keys, kst, m.klen, lane);
        }
      } else {
        const uint32_t from = head ? 0 : m.sh;
        if (part == 0) {  // header varints, key suffix, value length
          L.img[pos++] = (uint8_t)m.vt;
          pos = lds_put_leb(L.img, pos, m.seq);
          if (!head) pos = lds_put_leb(L.img, pos, m.sh);
          pos = lds_put_leb(L.img, pos, m.klen - from);
          lds_copy(L.img, pos, L.keys, kst + from, m.klen - from, lane);
          pos += m.klen - from;
          if (!is_tombstone(m.vt)) pos = lds_put_leb(L.img, pos, m.vl);
        }
        if (!is_tombstone(m.vt)) {  // the value: part q copies bytes [q vl / tpi, (q + 1) vl / tpi)
          uint32_t vpos = pos;
          if (part != 0)
            vpos = p0 + roff + 1 + leb_len(m.seq) + (head ? 0u : leb_len(m.sh)) + leb_len(m.klen - from) +
                   (m.klen - from) + leb_len(m.vl);
          const uint32_t va = (part * m.vl) >> tsh, vb = ((part + 1) * m.vl) >> tsh;
          lds_copy(L.img, vpos + va, L.vals, (uint32_t)(m.vo - vbase) + va, vb - va, lane);
        }
      }
      if (head && part == 0) {
        const uint32_t bp = p0 + B.recs + 1 + (m.e >> 16) * B.step;
        for (uint32_t q = 0; q < B.step; ++q) L.img[bp + q] = (uint8_t)(roff >> (8 * q));
      }
      if (kHash && B.hash_w && part == 0) {
        const uint32_t ridx = (item - B.it0) / ri;
        const uint32_t hb =
            kPlanBkt ? m.hb
                     : (uint32_t)(xxh3_64_any(m.klen, BaseReader8{L.keys, kst}, BaseReader64{L.keys, kst}) % B.hash_w);
        const uint32_t bk = B.hash_base + hb;
        atomicMin(&hlo[bk], ridx);
        atomicMax(&hhi[bk], ridx);
      }
    }
    }
    // ---- tails, wave per block: marker, hash-index bytes, trailer (trailer.rs:78-173);
    // without hash indexes they need nothing from the other waves' records
    // (disjoint bytes), so they go before the barrier
    auto tails = [&]() {
      for (uint32_t jb = wave; jb < (kDiagBuild && (P.diag & 8) ? 0 : k); jb += kGWaves) {
        const GBlk& B = TB[jb];
        const uint32_t p0 = B.img + kHdrLen, bin_off = B.recs + 1;
        if (lane == 0) L.img[p0 + B.recs] = kTrailerMarker;
        const uint32_t hash_off = B.hash_w ? bin_off + B.bin_len * B.step : 0;
        if (kHash)
          for (uint32_t q = lane; q < B.hash_w; q += kWave)
            L.img[p0 + hash_off + q] = (uint8_t)bucket_byte(hlo[B.hash_base + q], hhi[B.hash_base + q]);
        write_trailer_bytes(L.img, p0 + B.plen - kTrailerLen, ri, B.step, B.bin_len, bin_off, B.hash_w, hash_off,
                            B.n);
      }
    };
    if (!kHash) tails();
    group_barrier_lds();
    ENC_PHASE(3);
    // the stage is free: the next group's DMA runs under the tails and the hash
    if (Gn.k && !(kDiagBuild && (P.diag & 16))) issue_dma(Gn);
    ENC_PHASE(10);
    if (kHash) {  // the hash-index bytes need every vote
      tails();
      group_barrier_lds();
    }
    ENC_PHASE(4);
    // ---- payload xxh3_128: 1 KiB units over the 16 DPP rows
    {
      const uint32_t row = wave * 4 + (lane >> 4), r = lane & 15, q = r & 3, s = r >> 2;  // (4 kGWaves rows)
      const uint32_t ubase = rl32(r_upre, r0);
      const uint32_t units = (kDiagBuild && (P.diag & 10)) ? 0 : rl32(r_upre, r0 + k) - ubase;
      const uint64_t* acc = L.secret.acc + s + 2 * q;
      for (uint32_t u = row; u < units; u += 4 * kGWaves) {
        uint32_t jb = 0;  // (unit starts from the run registers: no dependent LDS reads)
        for (uint32_t x = 1; x < k; ++x) jb += (rl32(r_upre, r0 + x) - ubase <= u) ? 1u : 0u;
        const GBlk& B = TB[jb];
        const uint32_t n = u - B.u0, p0 = B.img + kHdrLen;
        uint64_t c0 = 0, c1 = 0;
        if (n < B.nbk) {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const Win16 w = read_win16(L.img, p0 + n * 1024 + 256 * t + 16 * r);
            stripe_part(w, acc[4 * t], acc[4 * t + 1], c0, c1);
          }
        } else {  // the tail stripes and the last stripe (secret + 121)
          const uint32_t tail0 = B.nbk * 1024, nb_stripes = ((B.plen - 1) - tail0) / 64;
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            if ((uint32_t)(4 * t + s) < nb_stripes) {
              const Win16 w = read_win16(L.img, p0 + tail0 + 256 * t + 16 * r);
              stripe_part(w, acc[4 * t], acc[4 * t + 1], c0, c1);
            }
          }
          if (r < 4) {
            const Win16 w = read_win16(L.img, p0 + B.plen - 64 + 16 * r);
            stripe_part(w, L.secret.last[2 * q], L.secret.last[2 * q + 1], c0, c1);
          }
        }
        c0 = row_quad_sum64(c0);
        c1 = row_quad_sum64(c1);
        if (r < 4) {
          contrib[8 * u + 2 * q] = c0;
          contrib[8 * u + 2 * q + 1] = c1;
        }
      }
    }
    group_barrier_lds();
    ENC_PHASE(5);
    // ---- one wave, a lane quad per block (k <= 16): the scramble chain and
    // the merge (or the short path), then the header.  Lane q of the quad
    // holds accumulator pair q; the chain is one instruction stream for all
    // the group's blocks.
    // The copy-out runs in two parts: the waves other than the chain wave store every whole
    // 16-B piece of the span that holds no header byte while the chain wave computes the
    // checksums and headers; after the barrier the header pieces (three per block) and the
    // partial pieces at both ends follow.  (Before, the whole copy-out waited for the chain.)
    const uint32_t cw = iter & (kGWaves - 1);  // the chain wave of this group
    const uint32_t total = (uint32_t)(rl64(r_off, r0 + k) - obase);
    const uint32_t end = (kDiagBuild && (P.diag & 4)) ? pad : pad + total;
    const uint32_t c0 = (pad + 15) >> 4, c1 = end >> 4;  // the whole 16-B pieces [c0, c1)
    const u32x4* const csrc = reinterpret_cast<const u32x4*>(L.img);
    u32x4* const cdst = reinterpret_cast<u32x4*>(dabs & ~15ULL);
    // the chain wave's header pieces
    const uint32_t hpc = (wave == cw && (uint32_t)lane < 3 * k) ? (TB[lane / 3].img >> 4) + lane % 3 : ~0u;
    if (wave == cw) {
      if (!(kDiagBuild && (P.diag & 10))) {
        const uint32_t jb = (uint32_t)lane >> 2;
        const int q = lane & 3;
        const bool in = jb < k;
        const GBlk& B = TB[in ? jb : 0];
        const uint32_t p0 = B.img + kHdrLen, plen = B.plen;
        uint64_t lo = 0, hi = 0;
        if (in && plen > 240) {
          uint64_t a0 = q == 0 ? (uint64_t)P32_3 : q == 1 ? P64_2 : q == 2 ? P64_4 : P64_5;
          uint64_t a1 = q == 0 ? P64_1 : q == 1 ? P64_3 : q == 2 ? (uint64_t)P32_2 : (uint64_t)P32_1;
          const uint64_t scr0 = L.secret.acc[16 + 2 * q], scr1 = L.secret.acc[16 + 2 * q + 1];
          const uint64_t* cb = contrib + 8 * B.u0 + 2 * q;
          // four KiB blocks' contributions per batch, read without branches (past
          // the block they read other contributions in L.uni, unused)
          for (uint32_t n0 = 0; n0 < B.nbk; n0 += 4) {
            uint64_t c0[4], c1[4];
#pragma unroll
            for (uint32_t t = 0; t < 4; ++t) {
              c0[t] = cb[8 * (n0 + t)];
              c1[t] = cb[8 * (n0 + t) + 1];
            }
#pragma unroll
            for (uint32_t t = 0; t < 4; ++t) {
              if (n0 + t < B.nbk) {
                a0 = xxh3_scr(a0, c0[t], scr0);
                a1 = xxh3_scr(a1, c1[t], scr1);
              }
            }
          }
          a0 += cb[8 * B.nbk];
          a1 += cb[8 * B.nbk + 1];
          lo = mul_fold64(a0 ^ L.secret.mlo[2 * q], a1 ^ L.secret.mlo[2 * q + 1]);
          hi = mul_fold64(a0 ^ L.secret.mhi[2 * q], a1 ^ L.secret.mhi[2 * q + 1]);
        }
        lo = quad_sum64(lo);  // (every lane: DPP reads of inactive lanes are undefined)
        hi = quad_sum64(hi);
        if (in) {
          if (plen > 240) {
            lo = xxh3_avalanche((uint64_t)plen * P64_1 + lo);
            hi = xxh3_avalanche(~((uint64_t)plen * P64_2) + hi);
          } else {
            xxh3_128_short(plen, BaseReader8{L.img, p0}, BaseReader64{L.img, p0}, lo, hi);
          }
          write_header_quad(L.img, B.img, P.type, lo, hi, plen, q);
          if (q == 0) P.status[G.b + jb] = ST_OK;
        }
      }
    } else {  // (no vmcnt wait here: the next group's DMA may still be landing)
      // the next group's block table, into the other buffer, by the wave after the chain wave
      if (Gn.k && wave == ((cw + 1) & (kGWaves - 1))) build_table(Gn, L.blk[(iter + 1) & 1]);
      const uint32_t t3 = ((wave + kGWaves - cw - 1) & (kGWaves - 1)) * kWave + (uint32_t)lane;  // 0 .. 191
      constexpr uint32_t kT3 = (kGWaves - 1) * kWave;
      // block j's header pieces are [hc_j, hc_j + 3) (33 bytes from any offset); its
      // header-free pieces run from hc_j + 3 to the next block's hc
      uint32_t hc = __builtin_amdgcn_readfirstlane(TB[0].img) >> 4;
      for (uint32_t jb = 0; jb < k; ++jb) {
        const uint32_t hn = jb + 1 < k ? __builtin_amdgcn_readfirstlane(TB[jb + 1].img) >> 4 : c1;
        for (uint32_t c = max(hc + 3, c0) + t3; c < min(hn, c1); c += kT3)
          *(__attribute__((address_space(1))) u32x4*)(cdst + c) = csrc[c];  // (plain stores, r06)
        hc = hn;
      }
    }
    group_barrier_lds();
    ENC_PHASE(6);
    __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0): the next group's DMA pieces and item fields
    ENC_PHASE(7);
    // ---- copy-out, part 2: the header pieces and the partial pieces at both ends
    {
      if (hpc >= c0 && hpc < c1) *(__attribute__((address_space(1))) u32x4*)(cdst + hpc) = csrc[hpc];
      // (shared with the neighbouring groups' bytes)
      auto* gb = (__attribute__((address_space(1))) uint8_t*)cdst;
      if (tid == 0)
        for (uint32_t x = pad; x < min(16 * c0, end); ++x) gb[x] = L.img[x];
      if (tid == kWave && c1 >= c0)
        for (uint32_t x = 16 * c1; x < end; ++x) gb[x] = L.img[x];
    }
    ENC_PHASE(8);
#ifdef LSM_DIAG
    ++ph_n;
#endif
    ++iter;
    G = Gn;
  }
#ifdef LSM_DIAG
  if ((P.diag & 0x80) && tid == 0) {
    for (int i = 0; i < 12; ++i) atomicAdd(&P.phase[i], (unsigned long long)ph_acc[i]);
    atomicAdd(&P.phase[15], (unsigned long long)ph_n);
  }
#endif
}

// Listed medium / big blocks: one wave per workgroup, grid-stride over the list.
template <int kOW>
__global__ __launch_bounds__(kWave) void encode_write_list_kernel(EncodeParams P, uint32_t plan_flag) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t count = P.list_count[0];
  for (uint32_t li = blockIdx.x; li < count; li += gridDim.x) {
    const uint32_t b = P.lists[li];
    if ((P.plans[b].step_flags >> 8) == plan_flag) write_block_lds<kOW>(P, b, smem);
  }
}

// Listed medium / big blocks, kLW waves per block (write_block_lds_mw).
template <uint32_t kLW, int kOW>
__global__ __launch_bounds__(kLW * kWave) void encode_write_list_mw_kernel(EncodeParams P, uint32_t plan_flag) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ uint32_t psum[kLW];
  __shared__ uint64_t contrib[8 * 64];
  const uint32_t count = P.list_count[0];
  for (uint32_t li = blockIdx.x; li < count; li += gridDim.x) {
    const uint32_t b = P.lists[li];
    if ((P.plans[b].step_flags >> 8) == plan_flag) write_block_lds_mw<kLW, kOW>(P, b, smem, psum, contrib);
  }
}

// ----------------------------------------------------- E3: HBM write pass
// Blocks larger than the list kernels' 96 KiB image (data blocks up to the
// writer's 4 MiB target, writer/mod.rs:193-198), one 8-wave workgroup per
// block, straight in HBM:
//   records  thread = item, at the record offset E1 left in erec (blocks of
//            more than kGItems items) or from a workgroup scan (fewer items);
//            the shared prefix is recomputed from the keys
//   hash     hash-index votes in LDS passes of kE3HashChunk buckets
//   tail     marker, trailer (wave 0)
//   xxh3     of the bytes just written: per 64 KiB, every wave reduces KiB
//            blocks into LDS contributions, then wave 0 carries the scramble
//            chain (as decode_chunked), the tail merge and the header.
constexpr uint32_t kE3Waves = 8, kE3Threads = kE3Waves * kWave;
template <int kOW>
__global__ __launch_bounds__(kE3Threads) void encode_large_kernel(EncodeParams P) {
  __shared__ uint32_t hlo[kE3HashChunk], hhi[kE3HashChunk];
  __shared__ uint64_t contrib[8 * 64];
  __shared__ uint32_t psum[kE3Waves];
  const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1);
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const uint32_t count = P.list_count[0];
  for (uint32_t li = blockIdx.x; li < count; li += gridDim.x) {
    const uint32_t b = P.lists[li];
    const BlockPlan pl = P.plans[b];
    if ((pl.step_flags >> 8) != kPlanHuge) continue;
    const uint32_t step = pl.step_flags & 0xFF;
    const uint64_t dst_off = P.block_off[b], dst_end = P.block_off[b + 1];
    if (dst_end > P.out_cap) {
      if (tid == 0) P.status[b] = ST_OVERFLOW;
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
    const bool scan = n <= kGItems;  // (uniform) else erec holds each record's offset
    const uint32_t pf = P.hb_sh ? P.pfirst[b] : 0u;  // (after E1p erec holds huge blocks' record prefixes)
    for (uint32_t j = tid; j < (scan ? kE3Threads : n); j += kE3Threads) {
      const bool head = j % ri == 0;
      ItemMeta m;
      uint32_t roff = 0;
      if (j < n) {
        bool bad = false;
        m = load_item_lcp<kOW>(P, s, j, ri, bad);
        if (!scan) roff = P.erec[s + j] - pf;  // (after E1p: the record prefix, see encode_e1p_offsets_kernel)
      }
      if (scan) {  // n <= kGItems <= kE3Threads: one pass
        const uint32_t rec = j < n ? (uint32_t)item_record_len(P, m, head) : 0u;
        const uint32_t incl = wave_incl_scan_u32(rec);
        if (lane == kWave - 1) psum[wave] = incl;
        __syncthreads();
        uint32_t base = 0;
        for (uint32_t w = 0; w < wave; ++w) base += psum[w];
        roff = base + incl - rec;
      }
      if (j < n) {
        RecordCopy rc;
        rc.issue(P, m, head, p0 + roff);
        rc.store(P, m, head, img);
        if (head) store_le(img, p0 + bin_off + (j / ri) * step, roff, step);
      }
    }
    const uint32_t hash_off = pl.hash_w ? bin_off + pl.bin_len * step : 0;
    for (uint32_t base = 0; base < pl.hash_w; base += kE3HashChunk) {
      const uint32_t lim = min(kE3HashChunk, pl.hash_w - base);
      for (uint32_t k = tid; k < lim; k += kE3Threads) {
        hlo[k] = 0xFFFFFFFFu;
        hhi[k] = 0;
      }
      __syncthreads();
      for (uint32_t j = tid; j < n; j += kE3Threads) {
        const uint64_t i = (uint64_t)s + j;
        const uint64_t ko = koff<kOW>(P, i);
        const uint32_t bk = key_bucket(P, ko, (uint32_t)(koff<kOW>(P, i + 1) - ko), pl.hash_w);
        if (bk >= base && bk < base + lim) {
          atomicMin(&hlo[bk - base], j / ri);
          atomicMax(&hhi[bk - base], j / ri);
        }
      }
      __syncthreads();
      for (uint32_t k = tid; k < lim; k += kE3Threads) img[p0 + hash_off + base + k] = (uint8_t)bucket_byte(hlo[k], hhi[k]);
      __syncthreads();
    }
    if (wave == 0) {
      if (lane == 0) img[p0 + pl.recs] = kTrailerMarker;
      write_trailer_bytes(img, p0 + plen - kTrailerLen, ri, step, pl.bin_len, bin_off, pl.hash_w, hash_off, n);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // the block's bytes, for this workgroup's re-reads below
    __syncthreads();
    uint64_t lo = 0, hi = 0;
    if (plen > 240) {
      const int q = lane & 3;
      uint64_t a0, a1;
      xxh3_acc_init(q, a0, a1);
      const uint64_t scr0 = kLongSecret.acc[16 + 2 * q], scr1 = kLongSecret.acc[16 + 2 * q + 1];
      const uint32_t nbk = (plen - 1) / 1024;
      for (uint32_t n0 = 0; n0 < nbk; n0 += 64) {
        const uint32_t n1 = min(nbk, n0 + 64);
        xxh3_kib_contribs<false>(img, p0 + 1024 * n0, (n1 - n0) * 1024 + 1, &kLongSecret, contrib, wave, kE3Waves);
        __syncthreads();
        if (wave == 0)
          for (uint32_t k = 0; k < n1 - n0; ++k) {
            a0 = xxh3_scr(a0, contrib[8 * k + 2 * q], scr0);
            a1 = xxh3_scr(a1, contrib[8 * k + 2 * q + 1], scr1);
          }
        __syncthreads();
      }
      if (wave == 0) xxh3_wave_tail_merge(img, p0, plen, &kLongSecret, a0, a1, lo, hi);
    } else if (wave == 0) {
      xxh3_128_wave(img, p0, plen, &kLongSecret, lo, hi);
    }
    if (wave == 0) {
      write_header_bytes(img, pad, P.type, lo, hi, plen);
      if (lane == 0) P.status[b] = ST_OK;
    }
    __syncthreads();
  }
}

// ---------------------------------------- E3 across the GPU (workspace pool)
// The one-workgroup E3 above writes a 1-4 MiB block's records with 512
// threads and carries its XXH3 chain on one wave, 64 KiB at a time.  With the
// pool (lsm_encode_workspace_size_ex) the huge blocks are collected by the
// size scan and cut into units any workgroup takes:
//   plan     (one workgroup) per collected block its record units, KiB-block
//            count and the prefix sums of both; accepted blocks are re-flagged
//            kPlanHugeGpu (the one-workgroup E3 passes them over)
//   records  record units of kEHugeItems items (thread per item at its E1
//            offset; blocks of <= kGItems items: one unit with a workgroup
//            scan), then one tail unit per block (hash-index votes, marker,
//            trailer)
//            (the contributions of the KiB blocks wholly inside a unit's LDS
//            image come from the image, flagged done)
//   chain    a workgroup per block: three waves hash the KiB blocks the
//            records kernel left into the pool while the fourth runs the eight
//            accumulator chains on lanes 0..7 behind them, then the tail merge,
//            the header and the status
constexpr uint32_t kEHugeItems = 1024;  // items per record unit, at most (four per thread)
constexpr uint32_t kEHugeImg = 2 * 4 * kE3HashChunk;  // LDS image of a record unit (the tail unit's vote arrays)
constexpr uint32_t kEHugeWgsPerCU = 4;  // encode_huge_records_kernel's residency (4 waves per SIMD, 32 KB of LDS)

struct EncHuge {
  uint64_t dst_off;
  uint64_t acc[8];
  uint32_t b, s, n, total;
  uint32_t nbk, nru, accepted, done;
  uint32_t ipu, pad;  // items per record unit
};
static_assert(sizeof(EncHuge) % 16 == 0, "EncHuge layout");
struct EncHugeHdr {
  uint64_t total_kib;
  uint32_t count;      // collected (atomic; may exceed the capacity: the rest stay with the one-workgroup E3)
  uint32_t n3;         // planned entries
  uint64_t total_units;
};
static_assert(offsetof(EncHugeHdr, count) == 4 * kEncHugeCountWord, "E1p clears the count by index");
// Pool: [hdr | 256][list u32 x cap][kpre u64 x (cap + 1)][upre u64 x (cap + 1)][EncHuge x cap]
// [contributions, 64 B per KiB block][done flags, 1 B per KiB block]
struct EncHugeLayout {
  EncHugeHdr* hdr;
  uint32_t* list;
  uint64_t* kpre;
  uint64_t* upre;
  EncHuge* rec;
  uint64_t* contrib;
  uint8_t* kdone;  // KiB block's contribution computed by the records kernel (from its LDS image)
  uint64_t cap_kib;
};
__host__ __device__ __forceinline__ uint64_t enc_huge_fixed_bytes(uint64_t cap) {
  return (256 + ((4 * cap + 15) & ~15ULL) + 16 * (cap + 1) + sizeof(EncHuge) * cap + 255) & ~255ULL;
}
__device__ __forceinline__ EncHugeLayout enc_huge_layout(const EncodeParams& P) {
  EncHugeLayout L;
  uint8_t* b = P.huge_pool;
  const uint64_t cap = P.huge_cap;
  L.hdr = reinterpret_cast<EncHugeHdr*>(b);
  L.list = reinterpret_cast<uint32_t*>(b + 256);
  L.kpre = reinterpret_cast<uint64_t*>(b + 256 + ((4 * cap + 15) & ~15ULL));
  L.upre = L.kpre + (cap + 1);
  L.rec = reinterpret_cast<EncHuge*>(L.upre + (cap + 1));
  const uint64_t fixed = enc_huge_fixed_bytes(cap);
  L.contrib = reinterpret_cast<uint64_t*>(b + fixed);
  L.cap_kib = (P.huge_pool_bytes - fixed) / 65;
  L.kdone = reinterpret_cast<uint8_t*>(L.contrib + 8 * L.cap_kib);
  return L;
}

__device__ __forceinline__ uint32_t last_le_u64(const uint64_t* a, uint32_t n, uint64_t v) {
  uint32_t lo = 0, hi = n;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a[mid] <= v) lo = mid;
    else hi = mid;
  }
  return lo;
}

// One workgroup of 1024 threads.
__global__ __launch_bounds__(1024) void encode_huge_plan_kernel(EncodeParams P) {
  __shared__ uint64_t sh[40];
  const EncHugeLayout L = enc_huge_layout(P);
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t n = min(L.hdr->count, P.huge_cap);
  if (tid == 0) sh[32] = 0, sh[33] = 0;
  __syncthreads();
  for (uint32_t c = 0; c < n; c += 1024) {
    const uint32_t i = c + tid;
    uint64_t nbk = 0, nu = 0;
    bool acc = false;
    EncHuge h{};
    if (i < n) {
      h.b = L.list[i];
      h.dst_off = P.block_off[h.b];
      const uint64_t dst_end = P.block_off[h.b + 1];
      h.s = P.starts[h.b];
      h.n = P.starts[h.b + 1] - h.s;
      h.total = (uint32_t)(dst_end - h.dst_off);
      acc = dst_end <= P.out_cap;  // (else the one-workgroup E3 reports the overflow)
      nbk = (h.total - kHdrLen - 1) / 1024;  // (payload > 96 KiB: the long path)
      // items per record unit: 7/8 of the LDS image at the block's mean record size (a unit over
      // the image goes straight to HBM and leaves its hash to the contrib kernel: the margin keeps
      // nearly every unit staged)
      const uint32_t recs = P.plans[h.b].recs;
      h.ipu = (uint32_t)min<uint64_t>(kEHugeItems, max<uint64_t>(64, (uint64_t)(kEHugeImg * 7 / 8) * h.n / max(recs, 1u)));
      h.nru = h.n <= kGItems ? 1 : (h.n + h.ipu - 1) / h.ipu;
      nu = acc ? h.nru + 1 : 0;
      nbk = acc ? nbk : 0;
    }
    const uint64_t ik = wave_incl_scan_u64(nbk), iu = wave_incl_scan_u64(nu);
    if (lane == 63) sh[wave] = ik, sh[16 + wave] = iu;
    __syncthreads();
    uint64_t bk = sh[32], bu = sh[33], tk = 0, tu = 0;
    for (uint32_t w = 0; w < 16; ++w) {
      bk += w < wave ? sh[w] : 0;
      bu += w < wave ? sh[16 + w] : 0;
      tk += sh[w];
      tu += sh[16 + w];
    }
    const uint64_t kp = bk + ik - nbk;
    if (i < n) {
      acc = acc && kp + nbk <= L.cap_kib;  // (the pool holds the contributions of a prefix of the list)
      h.nbk = (uint32_t)nbk;
      h.accepted = acc;
      h.done = 0;
      L.rec[i] = h;
      L.kpre[i] = kp;
      L.upre[i] = bu + iu - nu;
      if (acc) P.plans[h.b].step_flags = (P.plans[h.b].step_flags & 0xFF) | (kPlanHugeGpu << 8);
    }
    __syncthreads();
    if (tid == 0) sh[32] += tk, sh[33] += tu;
    __syncthreads();
  }
  if (tid == 0) {
    L.kpre[n] = sh[32];
    L.upre[n] = sh[33];
    L.hdr->total_kib = sh[32];
    L.hdr->total_units = sh[33];
    L.hdr->n3 = n;
  }
  // the records kernel's done flags start clear (the numbers of accepted blocks' KiB blocks are < cap_kib)
  const uint64_t nf = min(sh[32], L.cap_kib);
  for (uint64_t x = tid; 16 * x < nf; x += 1024) {
    if (16 * x + 16 <= nf) reinterpret_cast<u32x4*>(L.kdone)[x] = u32x4{0, 0, 0, 0};
    else
      for (uint64_t y = 16 * x; y < nf; ++y) L.kdone[y] = 0;
  }
}

// Record units (u < nru of a block) and the tail unit (u == nru).
template <int kOW>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void encode_huge_records_kernel(EncodeParams P) {
  __shared__ __attribute__((aligned(16))) uint32_t lbuf[2 * kE3HashChunk];  // record image | vote arrays
  uint32_t* hlo = lbuf;
  uint32_t* hhi = lbuf + kE3HashChunk;
  __shared__ uint32_t psum[4];
  const EncHugeLayout L = enc_huge_layout(P);
  const uint32_t n3 = L.hdr->n3;
  if (!n3) return;
  const uint64_t units = L.hdr->total_units;
  const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid >> 6;
  // a run of consecutive units per workgroup: one block search per run
  const uint64_t per = (units + gridDim.x - 1) / gridDim.x;
  const uint64_t u_begin = (uint64_t)blockIdx.x * per, u_end = min(units, u_begin + per);
  uint32_t i = u_begin < u_end ? last_le_u64(L.upre, n3, u_begin) : 0;
#ifdef LSM_DIAG  // diagnostic per-phase s_memtime totals of wave 0 (reserved bit 0x40)
  uint32_t ph_acc[8] = {}, ph_n = 0;
  uint64_t t_last = __builtin_amdgcn_s_memtime();
#define REC_PHASE(k)                                   \
  if (P.diag & 0x40) {                                 \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();  \
    ph_acc[k] += (uint32_t)(t_ - t_last);              \
    t_last = t_;                                       \
  }
#else
#define REC_PHASE(k)
#endif
  for (uint64_t u = u_begin; u < u_end; ++u) {
    REC_PHASE(6);
    while (i + 1 < n3 && gload(L.upre, i + 1) <= u) ++i;
    const EncHuge h = gload_pod(L.rec, i);
    if (!h.accepted) continue;  // (uniform; rejected blocks own no units)
    const uint32_t k = (uint32_t)(u - gload(L.upre, i));
    const BlockPlan pl = gload_pod(P.plans, h.b);
    const uint32_t step = pl.step_flags & 0xFF;
    const uint32_t ri = is_index(P) ? 1 : P.ri;
    const uint32_t plen = h.total - kHdrLen;
    const uint64_t dabs = (uint64_t)(uintptr_t)P.out + h.dst_off;
    uint8_t* img = reinterpret_cast<uint8_t*>(dabs & ~15ULL);
    const uint32_t p0 = (uint32_t)(dabs & 15) + kHdrLen;
    const uint32_t bin_off = pl.recs + 1;
    REC_PHASE(0);
    if (k < h.nru) {
      if (h.n <= kGItems) {  // one pass: record offsets from a workgroup scan
        const uint32_t j = tid;
        const bool head = j % ri == 0;
        ItemMeta m;
        bool bad = false;
        if (j < h.n) m = load_item_lcp<kOW>(P, h.s, j, ri, bad);
        const uint32_t rec = j < h.n ? (uint32_t)item_record_len(P, m, head) : 0u;
        const uint32_t incl = wave_incl_scan_u32(rec);
        if (lane == kWave - 1) psum[wave] = incl;
        __syncthreads();
        uint32_t base = 0;
        for (uint32_t w = 0; w < wave; ++w) base += psum[w];
        const uint32_t roff = base + incl - rec;
        if (j < h.n) {
          RecordCopy rc;
          rc.issue(P, m, head, p0 + roff);
          rc.store(P, m, head, as_gbl(img));
          if (head) store_le(as_gbl(img), p0 + bin_off + (j / ri) * step, roff, step);
        }
        __syncthreads();  // (psum is rewritten by the next unit)
      } else {
        // records [j0, j1) assembled in LDS (image bytes [a0, a0 + lend)), then copied
        // out in 16-B pieces; a unit larger than the image writes straight to HBM
        const uint32_t j0 = k * h.ipu, j1 = min(h.n, j0 + h.ipu);
        // (after E1p erec holds a huge block's record prefixes: offsets relative to its first)
        const uint32_t pf = P.hb_sh ? gload(P.pfirst, h.b) : 0u;
        const uint32_t rb = gload(P.erec, (uint64_t)h.s + j0) - pf;
        const uint32_t re = j1 < h.n ? gload(P.erec, (uint64_t)h.s + j1) - pf : pl.recs;
        const uint32_t a0 = (p0 + rb) & ~15u, lend = p0 + re - a0;
        const bool staged = lend + 32 <= kEHugeImg;  // (uniform)
        uint8_t* limg = reinterpret_cast<uint8_t*>(lbuf) - a0;  // image offset x -> LDS limg + x
        auto put = [&](auto* dst) {  // (two call sites: LDS and global stores)
          for (uint32_t j = j0 + tid; j < j1; j += 256) {
            const bool head = j % ri == 0;
            bool bad = false;
            // (after E1p the shared prefix is in hbucket: no key reads before the copy)
            ItemMeta m = P.hb_sh ? load_item<kOW>(P, (uint64_t)h.s + j, bad) : load_item_lcp<kOW>(P, h.s, j, ri, bad);
            if (P.hb_sh && !head) m.sh = gload(P.hbucket, (uint64_t)h.s + j);
            const uint32_t roff = gload(P.erec, (uint64_t)h.s + j) - pf;
            RecordCopy rc;
            rc.issue(P, m, head, p0 + roff);
            rc.store(P, m, head, dst);
            if (head) store_le(as_gbl(img), p0 + bin_off + (j / ri) * step, roff, step);
          }
        };
        if (staged) put(as_lds(limg));
        else put(as_gbl(img));
        REC_PHASE(1);
        if (staged) {
          __syncthreads();
          REC_PHASE(2);
          if (h.nbk) {  // the KiB blocks wholly inside these records: contributions from the image
            const uint32_t g0 = (rb + 1023) / 1024, g1 = min(h.nbk, re / 1024);
            if (g1 > g0) {
              const uint64_t kg = gload(L.kpre, i) + g0;
              xxh3_kib_contribs(reinterpret_cast<const uint8_t*>(lbuf), p0 + 1024 * g0 - a0, (g1 - g0) * 1024 + 1,
                                &kLongSecret, L.contrib + 8 * kg, wave, 4);  // (lbuf-relative: ds_read, not flat)
              for (uint32_t g = tid; g < g1 - g0; g += 256) L.kdone[kg + g] = 1;
            }
          }
          REC_PHASE(3);
          const uint32_t lo = (p0 + rb) - a0, c0 = (lo + 15) >> 4, c1 = lend >> 4;
          const u32x4* src = reinterpret_cast<const u32x4*>(lbuf);
          u32x4* dst = reinterpret_cast<u32x4*>(img + a0);
          for (uint32_t c = c0 + tid; c < c1; c += 256) copy_store16(dst + c, src[c]);
          // the partial pieces at both ends (shared with the neighbouring units' records)
          auto* gb = (__attribute__((address_space(1))) uint8_t*)(img + a0);
          const uint8_t* lb = reinterpret_cast<const uint8_t*>(lbuf);
          if (tid == 0)
            for (uint32_t x = lo; x < min(16 * c0, lend); ++x) gb[x] = lb[x];
          if (tid == kWave && c1 >= c0)
            for (uint32_t x = 16 * c1; x < lend; ++x) gb[x] = lb[x];
          __syncthreads();  // (the next unit rewrites the image)
          REC_PHASE(4);
        }
      }
#ifdef LSM_DIAG
      ++ph_n;
#endif
      continue;
    }
    // tail unit: hash-index votes (LDS passes), marker, trailer
    const uint32_t hash_off = pl.hash_w ? bin_off + pl.bin_len * step : 0;
    for (uint32_t base = 0; base < pl.hash_w; base += kE3HashChunk) {
      const uint32_t lim = min(kE3HashChunk, pl.hash_w - base);
      for (uint32_t q = tid; q < lim; q += 256) {
        hlo[q] = 0xFFFFFFFFu;
        hhi[q] = 0;
      }
      __syncthreads();
      for (uint32_t j = tid; j < h.n; j += 256) {
        const uint64_t it = (uint64_t)h.s + j;
        const uint64_t ko = koff<kOW>(P, it);
        const uint32_t bk = key_bucket(P, ko, (uint32_t)(koff<kOW>(P, it + 1) - ko), pl.hash_w);
        if (bk >= base && bk < base + lim) {
          atomicMin(&hlo[bk - base], j / ri);
          atomicMax(&hhi[bk - base], j / ri);
        }
      }
      __syncthreads();
      for (uint32_t q = tid; q < lim; q += 256) img[p0 + hash_off + base + q] = (uint8_t)bucket_byte(hlo[q], hhi[q]);
      __syncthreads();
    }
    if (wave == 0) {
      if (lane == 0) img[p0 + pl.recs] = kTrailerMarker;
      write_trailer_bytes(img, p0 + plen - kTrailerLen, ri, step, pl.bin_len, bin_off, pl.hash_w, hash_off, h.n);
    }
    REC_PHASE(5);
  }
#ifdef LSM_DIAG
  if ((P.diag & 0x40) && tid == 0) {
    for (int k = 0; k < 7; ++k) atomicAdd(&P.phase[k], (unsigned long long)ph_acc[k]);
    atomicAdd(&P.phase[15], (unsigned long long)ph_n);
  }
#endif
#undef REC_PHASE
}

// A four-wave workgroup per block.  Waves 1..3 hash the KiB blocks the records
// kernel left (kdone clear: across two record units, into the index / trailer,
// units over the LDS image, one-pass blocks) from the written payload: helper h
// takes the 64-row chunks h, h + 3, ... in order and publishes each in LDS.
// Wave 0 runs the eight accumulator chains on lanes 0..7 (xxh3_chain8), fetching
// a chunk's rows once its helper has published it, then the tail merge, the
// header (Header::encode_into) and the status.  The contributions cross a
// kernel boundary (an agent-scope fence per unit would write back the XCD's
// whole L2).
constexpr uint32_t kEChainRing = 16;
constexpr uint32_t kEChainHelpers = 3;
__global__ __launch_bounds__(256) void encode_huge_chain_kernel(EncodeParams P) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[kEChainRing * 1024];
  __shared__ uint32_t prog[4];  // helper h: 64-row chunks of this block done (h, h + 3, ... in order)
  const EncHugeLayout L = enc_huge_layout(P);
  const uint32_t n3 = L.hdr->n3;
  if (!n3) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63, k = lane & 7, q = lane & 3;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (tid < 4) prog[tid] = 0;
  __syncthreads();
  for (uint32_t i = blockIdx.x; i < n3; i += gridDim.x) {
    const EncHuge* r = L.rec + i;
    if (!r->accepted) continue;  // (uniform)
    const uint32_t nbk = r->nbk;
    const uint64_t kp = L.kpre[i];
    if (wave > 0) {
      const uint32_t h = wave - 1;
      const uint64_t dabs = (uint64_t)(uintptr_t)P.out + r->dst_off;
      const uint8_t* img = reinterpret_cast<const uint8_t*>(dabs & ~15ULL);
      const uint32_t p0 = (uint32_t)(dabs & 15) + kHdrLen;
      const uint64_t k0 = kLongSecret.acc[(lane >> 2) + 2 * q], k1 = kLongSecret.acc[(lane >> 2) + 2 * q + 1];
      uint32_t done = 0;
      for (uint32_t c = h; 64 * c < nbk; c += kEChainHelpers) {
        const uint32_t g = 64 * c + lane;
        uint64_t m = __ballot(g < nbk && !L.kdone[kp + g]);
        while (m) {  // four rows at a time (independent loads and sums)
          uint32_t gs[4];
          bool live[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            live[j] = m != 0;
            gs[j] = live[j] ? 64 * c + (uint32_t)__builtin_ctzll(m) : 64 * c;
            m &= m - 1;
          }
          Win16 w[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) w[j] = live[j] ? read_win16(img, p0 + 1024 * gs[j] + 16 * lane) : Win16{0, 0};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            uint64_t c0 = 0, c1 = 0;
            stripe_part(w[j], k0, k1, c0, c1);
            c0 = quad_group_sum64(c0);
            c1 = quad_group_sum64(c1);
            if (live[j] && lane < 4) {
              L.contrib[8 * (kp + gs[j]) + 2 * q] = c0;
              L.contrib[8 * (kp + gs[j]) + 2 * q + 1] = c1;
            }
          }
        }
        vm_wait<0>();  // (the rows' stores, before the chain wave's DMA reads them)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_store(&prog[h], ++done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      __syncthreads();  // (the chain wave's end of this block)
      __syncthreads();
      continue;
    }
    uint64_t a0, a1;
    xxh3_acc_init((int)(k >> 1), a0, a1);
    uint64_t x = (k & 1) ? a1 : a0;
    // chunk qq of 16 rows lies in 64-row chunk qq / 4, helper (qq / 4) % 3's (qq / 4) / 3 + 1-th
    auto wait = [&](uint64_t qq) {
      const uint32_t c = (uint32_t)(qq / 4);
      while (__hip_atomic_load(&prog[c % kEChainHelpers], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <
             c / kEChainHelpers + 1)
        __builtin_amdgcn_s_sleep(1);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    };
    if (nbk) x = xxh3_chain8<kEChainRing>(L.contrib + 8 * kp, nbk, x, kLongSecret.acc[16 + k], ring, wait);
    // lane quad position q takes accumulators 2q, 2q + 1 (lanes 2q, 2q + 1 hold them)
    const uint64_t c0 = wave_shfl_u64(x, (int)(2 * q)), c1 = wave_shfl_u64(x, (int)(2 * q + 1));
    const uint64_t dabs = (uint64_t)(uintptr_t)P.out + r->dst_off;
    uint8_t* img = reinterpret_cast<uint8_t*>(dabs & ~15ULL);
    const uint32_t pad = (uint32_t)(dabs & 15), plen = r->total - kHdrLen;
    uint64_t lo, hi;
    xxh3_wave_tail_merge(img, pad + kHdrLen, plen, &kLongSecret, c0, c1, lo, hi);
    write_header_bytes(img, pad, P.type, lo, hi, plen);
    if (lane == 0) P.status[r->b] = ST_OK;
    __syncthreads();  // every helper is past its last chunk of this block
    if (lane < 4) prog[lane] = 0;
    __syncthreads();
  }
}

// The size scan's outputs: block offsets (low 40 bits of the prefix) and the
// list of the listed blocks (high bits = their running count); with the pool,
// the huge blocks are also collected (hdr->count) for the whole-GPU E3.
struct EncodeOffOut {
  uint64_t* off;
  const uint64_t* sizes;
  uint32_t* list;
  uint32_t* count;
  uint64_t n;
  const BlockPlan* plans;
  uint32_t* huge_count;  // null: no pool
  uint32_t* huge_list;
  uint32_t huge_cap;
};

// The size scan's apply pass (scan_tile_apply's shape, the outputs above): a
// thread's kScanPerThread sizes, and for its listed blocks their plan flags,
// are all read before the scan; the huge blocks take their list slots from one
// atomic per wave (a per-block atomic on one counter serialised a batch of 240
// huge blocks at 7.8 us).
__global__ __launch_bounds__(kScanThreads) void encode_offsets_apply_kernel(const uint64_t* __restrict__ tile_offsets,
                                                                            EncodeOffOut o) {
  __shared__ uint64_t sh[kScanThreads / 64];
  const uint64_t n = o.n;
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanPerThread;
  const uint32_t lane = threadIdx.x & (kWave - 1);
  uint64_t v[kScanPerThread];
  scan_load(o.sizes, base, n, v);
  bool huge[kScanPerThread];
  uint32_t hc = 0;
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < kScanPerThread; ++i) {
    huge[i] = o.huge_count && base + i < n && (v[i] & ~kOffMask) &&
              (o.plans[base + i].step_flags >> 8) == kPlanHuge;
    hc += huge[i] ? 1u : 0u;
    s += v[i];
  }
  uint64_t total;
  uint64_t ex = block_excl_scan_u64(s, sh, total) + (tile_offsets ? tile_offsets[blockIdx.x] : 0);
  uint32_t slot = 0;
  if (o.huge_count) {  // (uniform)
    const uint32_t incl = wave_incl_scan_u32(hc);
    const uint32_t wtot = (uint32_t)__shfl((int)incl, kWave - 1);
    uint32_t wb = 0;
    if (lane == 0 && wtot) wb = atomicAdd(o.huge_count, wtot);
    slot = (uint32_t)__shfl((int)wb, 0) + incl - hc;
  }
#pragma unroll
  for (int i = 0; i < kScanPerThread; ++i) {
    const uint64_t k = base + i;
    if (k < n) {
      o.off[k] = ex & kOffMask;
      if (v[i] & ~kOffMask) o.list[ex >> 40] = (uint32_t)k;
      if (huge[i]) {
        if (slot < o.huge_cap) o.huge_list[slot] = (uint32_t)k;
        ++slot;
      }
    }
    if (k == n - 1) {
      o.off[n] = (ex + v[i]) & kOffMask;
      *o.count = (uint32_t)((ex + v[i]) >> 40);
    }
    ex += v[i];
  }
}

#ifdef LSM_DIAG
static unsigned long long* diag_phase_buffer() {
  static unsigned long long* d = nullptr;
  if (!d && hipMalloc(&d, 16 * sizeof(unsigned long long)) == hipSuccess) (void)hipMemset(d, 0, 16 * sizeof(unsigned long long));
  return d;
}
#endif

static size_t al256(size_t x) { return (x + 255) / 256 * 256; }

// A plan workgroup walks its blocks' items serially (chunks of 512), so it
// owns about 16 Ki items: kPlanBlocks blocks of the 4 KiB shapes, down to one
// block each for 1-4 MiB data blocks (which gave a single workgroup 3 M items
// and a 27 ms plan for 60 blocks of 4 MiB).
static uint32_t plan_blocks_per_wg(uint64_t n_items, uint32_t n_blocks) {
  const uint64_t avg = n_blocks ? (n_items + n_blocks - 1) / n_blocks : 1;
  const uint64_t bpw = (16384 + avg - 1) / (avg ? avg : 1);
  return (uint32_t)std::min<uint64_t>(kPlanBlocks, std::max<uint64_t>(1, bpw));
}

// kspan, vspan | sizes | plans | lists | list count + E1p flag | scan tiles (blocks or items) |
// erec | hbucket | hb_fix | pfirst | wpart
static uint64_t enc_tiles(uint64_t n_items, uint32_t n_blocks) {
  return std::max<uint64_t>(scan_tiles(n_blocks), scan_tiles(std::max<uint64_t>(n_items, 1)));
}
size_t encode_workspace_size(uint64_t n_items, uint32_t n_blocks) {
  return 2 * al256(((size_t)n_blocks + 1) * 8) + al256((size_t)n_blocks * 8) +
         al256((size_t)n_blocks * sizeof(BlockPlan)) + al256((size_t)n_blocks * 4) + 256 +
         al256(enc_tiles(n_items, n_blocks) * 8) + al256((size_t)n_items * 4) + al256((size_t)n_items * 2) + 256 +
         al256(((size_t)n_blocks + 1) * 4) + al256((n_items / 64 + 1) * 16);
}

// Huge-list entries for an output of out_cap bytes: a huge block's image
// exceeds kImgBig, so its encoded bytes exceed 32 KiB (entries past the
// capacity stay with the one-workgroup E3).
static uint64_t enc_huge_cap(uint32_t n_blocks, uint64_t out_cap) {
  return std::min<uint64_t>(n_blocks, out_cap / 32768 + 1);
}

size_t encode_workspace_size_ex(uint64_t n_items, uint32_t n_blocks, uint64_t out_cap) {
  const size_t ex = encode_workspace_size(n_items, n_blocks) + enc_huge_fixed_bytes(enc_huge_cap(n_blocks, out_cap)) +
                    65 * (out_cap / 1024 + 1) + 256;
  return std::max(ex, encode_pool_min_bytes(n_items, n_blocks, out_cap));
}

size_t encode_pool_min_bytes(uint64_t n_items, uint32_t n_blocks, uint64_t out_cap) {
  return al256(encode_workspace_size(n_items, n_blocks)) + enc_huge_fixed_bytes(enc_huge_cap(n_blocks, out_cap)) +
         65 * 128;
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
                         int32_t* status, void* ws, size_t ws_bytes, hipStream_t st, bool off32) {
  EncodeParams P;
  P.it = items;
  P.off32 = off32 ? 1u : 0u;
  P.starts = starts;
  P.n_blocks = n_blocks;
  P.ri = params.block_type == 1 ? 1 : params.restart_interval;
  P.ratio = params.block_type == 1 ? 0.0f : params.hash_ratio;
  P.type = params.block_type;
  P.diag = params.reserved;
#ifdef LSM_DIAG
  P.phase = diag_phase_buffer();
#else
  P.phase = nullptr;
#endif
  P.out = out;
  P.out_cap = out_cap;
  P.block_off = block_off;
  P.status = status;
  uint8_t* w = (uint8_t*)ws;
  P.kspan = (uint64_t*)w; w += al256(((size_t)n_blocks + 1) * 8);
  P.vspan = (uint64_t*)w; w += al256(((size_t)n_blocks + 1) * 8);
  P.sizes = (uint64_t*)w; w += al256((size_t)n_blocks * 8);
  P.plans = (BlockPlan*)w; w += al256((size_t)n_blocks * sizeof(BlockPlan));
  P.lists = (uint32_t*)w; w += al256((size_t)n_blocks * 4);
  P.list_count = (uint32_t*)w;
  P.e1p_flag = (uint32_t*)w + 1;
  w += 256;
  uint64_t* tiles = (uint64_t*)w; w += al256(enc_tiles(items.n_items, n_blocks) * 8);
  P.erec = (uint32_t*)w; w += al256((size_t)items.n_items * 4);
  P.hbucket = (uint16_t*)w; w += al256((size_t)items.n_items * 2);
  P.hb_fix = (uint32_t*)w; w += 256;
  P.pfirst = (uint32_t*)w; w += al256(((size_t)n_blocks + 1) * 4);
  P.wpart = (uint64_t*)w;
  hipError_t e;
  P.plan_bpw = plan_blocks_per_wg(items.n_items, n_blocks);
  P.hb_valid = 0;
  P.hb_sh = 0;
  const dim3 pgrid((n_blocks + P.plan_bpw - 1) / P.plan_bpw);
  const bool e1p = P.type != 1 && P.plan_bpw <= kE1pMaxBpw && items.n_items > 0 && items.n_items < 0xFFFFFFFFull;
  {  // the whole-GPU E3 pool, when the caller asks for it (the ABI checked the size)
    const size_t base = al256(encode_workspace_size(items.n_items, n_blocks));
    const uint64_t cap = enc_huge_cap(n_blocks, out_cap);
    const bool pool = cap && (params.flags & LSM_ENCODE_HUGE_POOL) &&
                      ws_bytes >= encode_pool_min_bytes(items.n_items, n_blocks, out_cap);
    P.huge_pool = pool ? (uint8_t*)ws + base : nullptr;
    P.huge_pool_bytes = pool ? ws_bytes - base : 0;
    P.huge_cap = pool ? (uint32_t)cap : 0;
    // (E1p's lengths kernel writes the E1p flag whole and clears the huge-block count:
    // no clear launch; otherwise the pool header is cleared here)
    if (pool && !e1p && (e = fill_words_async(P.huge_pool, 64, 0, st)) != hipSuccess) return e;
  }
  // The run-level plan fused into the group kernel (decoupled look-back for the offsets):
  // data blocks without a hash index, up to 512 items per block on average, no pool, and
  // fewer than 2^21 blocks (the listed count's bits in a look-back word); asked for
  // (LSM_ENCODE_RUN_PLAN) or at >= kFusedAutoItems items per block on average, where it
  // measured faster (profiles/r06_experiments.txt, ab6h / ab6i).
#ifdef LSM_NO_FUSED_PLAN
  constexpr bool kFusedOk = false;
#else
  constexpr bool kFusedOk = true;
#endif
  const uint64_t avg_items = n_blocks ? items.n_items / n_blocks : 0;
  const bool fused = kFusedOk && !e1p && P.type != 1 && !(P.ratio > 0.0f) && !P.huge_pool && P.plan_bpw >= 32 &&
                     n_blocks > 0 && n_blocks < (1u << 21) &&
                     ((params.flags & LSM_ENCODE_RUN_PLAN) || avg_items >= kFusedAutoItems);
  if (fused) {  // the look-back words (P.sizes, unused by this path) start cleared
    if ((e = fill_words_grid_async(P.sizes, 2 * ((n_blocks + kGRunFused - 1) / kGRunFused), 0, st)) != hipSuccess)
      return e;
  } else if (e1p) {  // batches of huge blocks: the plan item-parallel
    P.hb_sh = 1;
    const dim3 igrid((uint32_t)((items.n_items + 256 * kE1pPer - 1) / (256 * kE1pPer)));
    const dim3 lgrid((uint32_t)((items.n_items + 256 * kE1pLenPer - 1) / (256 * kE1pLenPer)));
    if (P.off32) hipLaunchKernelGGL(encode_e1p_lengths_kernel<4>, lgrid, dim3(256), 0, st, P);
    else hipLaunchKernelGGL(encode_e1p_lengths_kernel<8>, lgrid, dim3(256), 0, st, P);
    if ((e = launch_excl_scan(P.erec, items.n_items, tiles, E1pOut{P.erec, P.pfirst + n_blocks, items.n_items},
                              st)) != hipSuccess)
      return e;
    hipLaunchKernelGGL(encode_e1p_blocks_kernel, dim3((uint32_t)(((uint64_t)n_blocks + 3) / 4)), dim3(256), 0, st, P);
    hipLaunchKernelGGL(encode_e1p_offsets_kernel, igrid, dim3(256), 0, st, P);
  } else if (P.type == 1)
    hipLaunchKernelGGL(encode_plan_kernel<true>, pgrid, dim3(256), 0, st, P);
  // (the wave kernel gives each wave whole blocks: with a few blocks of many items
  // per workgroup most waves would idle, so those batches keep the workgroup walk)
  else if (P.plan_bpw >= 16 && P.ratio > 0.0f) {  // (only this plan kernel fills hbucket)
    P.hb_valid = 1;
    if ((e = fill_words_async(P.hb_fix, 1, 0, st)) != hipSuccess) return e;
    if (P.off32) hipLaunchKernelGGL((encode_plan_wave_kernel<true, 4>), pgrid, dim3(256), 0, st, P);
    else hipLaunchKernelGGL((encode_plan_wave_kernel<true, 8>), pgrid, dim3(256), 0, st, P);
    hipLaunchKernelGGL(encode_bucket_fixup_kernel, dim3(1024), dim3(256), 0, st, P);
  } else if (P.plan_bpw >= 16)
    if (P.off32) hipLaunchKernelGGL((encode_plan_wave_kernel<false, 4>), pgrid, dim3(256), 0, st, P);
    else hipLaunchKernelGGL((encode_plan_wave_kernel<false, 8>), pgrid, dim3(256), 0, st, P);
  else
    hipLaunchKernelGGL(encode_plan_kernel<false>, pgrid, dim3(256), 0, st, P);
  EncodeOffOut oo{block_off, P.sizes, P.lists, P.list_count, n_blocks, P.plans, nullptr, nullptr, 0};
  if (P.huge_pool) {
    oo.huge_count = &reinterpret_cast<EncHugeHdr*>(P.huge_pool)->count;
    oo.huge_list = reinterpret_cast<uint32_t*>(P.huge_pool + 256);
    oo.huge_cap = P.huge_cap;
  }
  if (!fused) {
    const uint64_t* offs;
    if ((e = launch_scan_tile_offsets(P.sizes, n_blocks, tiles, st, &offs)) != hipSuccess) return e;
    hipLaunchKernelGGL(encode_offsets_apply_kernel, dim3((uint32_t)scan_tiles(n_blocks)), dim3(kScanThreads), 0, st,
                       offs, oo);
  }
  // (the cold kernels too are instantiated per offset width: a run-time width branch per
  // item load cost the 1 / 4 MiB encodes 5-6 %, profiles/r06_experiments.txt)
  const bool w4 = P.off32 != 0;
  const void* list_k = w4 ? (const void*)encode_write_list_kernel<4> : (const void*)encode_write_list_kernel<8>;
  const void* list_mw_k = w4 ? (const void*)encode_write_list_mw_kernel<kListBigWaves, 4>
                             : (const void*)encode_write_list_mw_kernel<kListBigWaves, 8>;
  static uint64_t attr_done[2] = {0, 0}, attr_mw[2] = {0, 0};
  if ((e = set_lds_attr(list_k, kImgBig, &attr_done[w4])) != hipSuccess) return e;
  if ((e = set_lds_attr(list_mw_k, kImgBig, &attr_mw[w4])) != hipSuccess) return e;
  const dim3 ggrid((n_blocks + kGRun - 1) / kGRun), gblock(kGThreads);
  // (kernels instantiated per offset width: straight-line item loads)
  if (P.type == 1)
    hipLaunchKernelGGL(w4 ? (encode_group_kernel<true, false, false, 4>) : (encode_group_kernel<true, false, false, 8>),
                       ggrid, gblock, 0, st, P);
  else if (P.ratio > 0.0f && P.hb_valid)  // buckets from the plan pass
    hipLaunchKernelGGL(w4 ? (encode_group_kernel<false, true, true, 4>) : (encode_group_kernel<false, true, true, 8>),
                       ggrid, gblock, 0, st, P);
  else if (P.ratio > 0.0f)
    hipLaunchKernelGGL(w4 ? (encode_group_kernel<false, true, false, 4>) : (encode_group_kernel<false, true, false, 8>),
                       ggrid, gblock, 0, st, P);
  else if (fused)
    hipLaunchKernelGGL(w4 ? (encode_group_kernel<false, false, false, 4, true>)
                          : (encode_group_kernel<false, false, false, 8, true>),
                       dim3((n_blocks + kGRunFused - 1) / kGRunFused), gblock, 0, st, P);
  else
    hipLaunchKernelGGL(w4 ? (encode_group_kernel<false, false, false, 4>) : (encode_group_kernel<false, false, false, 8>),
                       ggrid, gblock, 0, st, P);
  // medium blocks (<= 20 KiB images): one wave each, eight workgroups per CU, was
  // faster than four waves each (2.26 vs 2.40 ms for the 16 KiB random-key class)
  if (w4) {
    hipLaunchKernelGGL(encode_write_list_kernel<4>, dim3(2048), dim3(kWave), kImgMedium, st, P, kPlanMedium);
    hipLaunchKernelGGL((encode_write_list_mw_kernel<kListBigWaves, 4>), dim3(512), dim3(kListBigWaves * kWave),
                       kImgBig, st, P, kPlanBig);
  } else {
    hipLaunchKernelGGL(encode_write_list_kernel<8>, dim3(2048), dim3(kWave), kImgMedium, st, P, kPlanMedium);
    hipLaunchKernelGGL((encode_write_list_mw_kernel<kListBigWaves, 8>), dim3(512), dim3(kListBigWaves * kWave),
                       kImgBig, st, P, kPlanBig);
  }
  if (P.huge_pool) {  // huge blocks across the GPU (the ones it does not take stay flagged for E3 below)
    hipLaunchKernelGGL(encode_huge_plan_kernel, dim3(1), dim3(1024), 0, st, P);
    // one resident wave of record workgroups (no partly filled last wave: 256 KiB encode
    // 0.459 -> 0.424 ms against a 2048-workgroup grid)
    static int cu_count[64] = {};  // per device (benign race: every writer stores the same count)
    int dev = 0;
    if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
    int n_cu = dev < 64 ? __atomic_load_n(&cu_count[dev], __ATOMIC_RELAXED) : 0;
    if (!n_cu) {
      if ((e = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
      if (dev < 64) __atomic_store_n(&cu_count[dev], n_cu, __ATOMIC_RELAXED);
    }
    const dim3 rgrid(kEHugeWgsPerCU * (uint32_t)n_cu);
    if (w4) hipLaunchKernelGGL(encode_huge_records_kernel<4>, rgrid, dim3(256), 0, st, P);
    else hipLaunchKernelGGL(encode_huge_records_kernel<8>, rgrid, dim3(256), 0, st, P);
    hipLaunchKernelGGL(encode_huge_chain_kernel, dim3(min(n_blocks, 1024u)), dim3(256), 0, st, P);
  }
  if (w4) hipLaunchKernelGGL(encode_large_kernel<4>, dim3(512), dim3(kE3Threads), 0, st, P);
  else hipLaunchKernelGGL(encode_large_kernel<8>, dim3(512), dim3(kE3Threads), 0, st, P);
  return hipGetLastError();
}

}  // namespace lsmgpu

#ifdef LSM_DIAG
// Diagnostic builds only: copy out and clear the per-phase cycle totals.
extern "C" int lsm_diag_encode_phases(uint64_t* out16) {
  unsigned long long* d = lsmgpu::diag_phase_buffer();
  if (!d || hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpy(out16, d, 16 * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return hipMemset(d, 0, 16 * sizeof(uint64_t)) == hipSuccess ? 0 : -1;
}
#endif
