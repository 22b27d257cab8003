// decode.hip — batched SST block decode on gfx950 (the north-star hot path).
//
// Replaces, per block, Block::from_file (header decode + xxh3_128 verify,
// src/table/block/mod.rs:131-182), the load_block type check
// (src/table/util.rs:79-86) and the full forward DataBlock::iter() /
// IndexBlock::iter() (src/table/block/decoder.rs:442-483) over a whole batch.
//
// Launch shape (DESIGN.md "Decode kernel"):
//   * one 64-lane wave per workgroup; wave w owns blocks [w*BPW, (w+1)*BPW);
//   * it repeatedly takes the longest run of its next blocks that fits the
//     LDS stage (stage_bytes) and the output tile (tile_items), copies the
//     run's bytes HBM->LDS in one coalesced 16 B/lane sweep (consecutive
//     blocks are contiguous on disk, so a run is one contiguous span);
//   * header checks run lane-parallel (lane j = block j of the run);
//   * each payload's xxh3_128 is computed by the whole wave from LDS;
//   * restart intervals are the unit of parallelism: lane = (block, restart),
//     each lane walks its interval's records with a 16-byte register window;
//   * parsed items land in an LDS SoA tile and leave in coalesced stores.
// Blocks larger than the stage run the same code directly on HBM.
#include <hip/hip_runtime.h>

#include "block_format.hpp"
#include "decode.hpp"
#include "scan.hpp"

namespace lsmgpu {

struct alignas(16) BlockMeta {
  uint64_t ck_lo, ck_hi;
  uint32_t hb;        // byte offset of the header in the image / span
  uint32_t len;       // handle size (header + payload)
  int32_t st;         // lsm_status
  uint32_t type;
  uint32_t ri, step, bin_len, bin_off, item_count, rec_end;
  uint32_t item0;     // first output index relative to the group base
  uint32_t chain0;    // exclusive prefix of restart intervals in the group
};
constexpr uint32_t kMetaBytes = 64 * sizeof(BlockMeta);

struct TileView {
  uint64_t* seqno;
  uint32_t *key_off, *val_off, *val_len;
  uint16_t *key_len, *prefix_len;
  uint8_t* vtype;
};

__host__ __device__ constexpr uint32_t tile_bytes(uint32_t items) {
  // each array 16-byte aligned
  return ((items * 8 + 15) & ~15u) + 3 * ((items * 4 + 15) & ~15u) + 2 * ((items * 2 + 15) & ~15u) +
         ((items + 15) & ~15u);
}
__device__ __forceinline__ TileView make_tile(uint8_t* t, uint32_t items) {
  TileView v;
  v.seqno = (uint64_t*)t; t += (items * 8 + 15) & ~15u;
  v.key_off = (uint32_t*)t; t += (items * 4 + 15) & ~15u;
  v.val_off = (uint32_t*)t; t += (items * 4 + 15) & ~15u;
  v.val_len = (uint32_t*)t; t += (items * 4 + 15) & ~15u;
  v.key_len = (uint16_t*)t; t += (items * 2 + 15) & ~15u;
  v.prefix_len = (uint16_t*)t; t += (items * 2 + 15) & ~15u;
  v.vtype = (uint8_t*)t;
  return v;
}

__device__ __forceinline__ void emit_tile(const TileView& t, uint32_t i, const ItemFields& f) {
  t.seqno[i] = f.seqno;
  t.key_off[i] = f.key_off;
  t.val_off[i] = f.val_off;
  t.val_len[i] = f.val_len;
  t.key_len[i] = f.key_len;
  t.prefix_len[i] = f.prefix_len;
  t.vtype[i] = f.vtype;
}
__device__ __forceinline__ void emit_global(const lsm_parsed_items& o, uint64_t i, const ItemFields& f) {
  if (o.seqno) o.seqno[i] = f.seqno;
  if (o.key_off) o.key_off[i] = f.key_off;
  if (o.val_off) o.val_off[i] = f.val_off;
  if (o.val_len) o.val_len[i] = f.val_len;
  if (o.key_len) o.key_len[i] = f.key_len;
  if (o.prefix_len) o.prefix_len[i] = f.prefix_len;
  if (o.vtype) o.vtype[i] = f.vtype;
  if (o.handle_off) o.handle_off[i] = f.handle_off;
}

// Lane-level: header + (after the wave hash) trailer checks, oracle order.
__device__ __forceinline__ void meta_header(const uint8_t* base, uint32_t hb, uint64_t len, BlockMeta& m) {
  HeaderInfo h;
  m.hb = hb;
  m.len = (uint32_t)len;
  m.st = (len > 0xFFFFFF00ULL) ? ST_TRUNCATED : check_header(base, hb, len, h);
  if (m.st == ST_OK) {
    m.ck_lo = h.ck_lo;
    m.ck_hi = h.ck_hi;
    m.type = h.type;
    m.item_count = h.data_length;  // stash data_length until meta_trailer
  }
  m.chain0 = 0;
}

__device__ __forceinline__ void meta_trailer(const uint8_t* base, int32_t expect_type, uint32_t cap, BlockMeta& m) {
  if (m.st != ST_OK) return;
  const uint32_t plen = m.len - kHdrLen;
  if (m.item_count != plen) { m.st = ST_TRUNCATED; return; }   // data_length vs handle
  if (expect_type >= 0 && (int32_t)m.type != expect_type) { m.st = ST_TYPE_MISMATCH; return; }
  if (m.type == 2) { m.st = ST_UNSUPPORTED; return; }          // filter blocks are not KV blocks
  TrailerInfo t;
  int32_t st = read_trailer(base, m.hb + kHdrLen, plen, t);
  if (st == ST_OK && m.type == 1 && t.ri != 1) st = ST_PARSE;   // index blocks: restart interval 1
  if (st == ST_OK && t.item_count > cap) st = ST_OVERFLOW;
  m.st = st;
  if (st != ST_OK) return;
  m.ri = t.ri; m.step = t.step; m.bin_len = t.bin_len; m.bin_off = t.bin_off;
  m.item_count = t.item_count; m.rec_end = t.rec_end;
}

// Walk restart interval r of a block whose payload starts at base[p0].
// Emits through `emit(j, fields)` with j = item index within the block.
template <class Emit>
__device__ __forceinline__ bool walk_interval(const uint8_t* base, uint32_t p0, const BlockMeta& m, uint32_t r,
                                              Emit emit) {
  TrailerInfo t;
  t.ri = m.ri; t.step = m.step; t.bin_len = m.bin_len; t.bin_off = m.bin_off;
  t.item_count = m.item_count; t.rec_end = m.rec_end;
  const bool last = r + 1 == t.bin_len;
  const uint32_t start = bin_get(base, p0, t, r);
  const uint32_t stop = last ? t.rec_end : bin_get(base, p0, t, r + 1);
  const uint32_t count = last ? t.item_count - r * t.ri : t.ri;
  if (start > t.rec_end || stop > t.rec_end) return false;
  Cursor c;
  c.init(base, p0, start, t.rec_end);
  ItemFields f;
  if (m.type == 1) {
    if (!parse_index_record(c, f)) return false;
    emit(r, f);
  } else {
    uint32_t base_key = 0;
    for (uint32_t j = 0; j < count; ++j) {
      if (!parse_data_record(c, j == 0, base_key, f)) return false;
      if (j == 0) base_key = f.key_off;
      emit(r * t.ri + j, f);
    }
  }
  return c.pos == stop;
}

// One block straight from HBM (blocks larger than the LDS stage).
__device__ void decode_block_direct(const DecodeParams& P, uint32_t b, BlockMeta* meta) {
  const int lane = threadIdx.x;
  const uint64_t off = P.block_off[b], end = P.block_off[b + 1];
  const uint8_t* base = P.blocks + (off & ~15ULL);
  const uint32_t hb = (uint32_t)(off & 15);
  const uint64_t len = end >= off ? end - off : 0;
  const uint64_t item_base = P.item_start[b];
  const uint32_t cap = P.item_start[b + 1] - P.item_start[b];
  if (lane == 0) meta_header(base, hb, len, meta[0]);
  __syncthreads();
  if (meta[0].st == ST_OK) {
    uint64_t lo, hi;
    xxh3_128_wave(base, hb + kHdrLen, meta[0].len - kHdrLen, &kLongSecret, lo, hi);
    if (lane == 0 && (lo != meta[0].ck_lo || hi != meta[0].ck_hi)) meta[0].st = ST_CKSUM;
  }
  __syncthreads();
  if (lane == 0) meta_trailer(base, P.expect_type, cap, meta[0]);
  __syncthreads();
  const BlockMeta m = meta[0];
  if (m.st == ST_OK) {
    bool ok = true;
    for (uint32_t r = lane; r < m.bin_len; r += kWave) {
      ok &= walk_interval(base, hb + kHdrLen, m, r,
                          [&](uint32_t j, const ItemFields& f) { emit_global(P.out, item_base + j, f); });
    }
    if (!ok) atomicCAS(&meta[0].st, ST_OK, ST_PARSE);
  }
  __syncthreads();
  if (lane == 0) P.status[b] = meta[0].st;
  __syncthreads();
}

__global__ __launch_bounds__(64) void decode_blocks_kernel(DecodeParams P) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  BlockMeta* meta = reinterpret_cast<BlockMeta*>(smem);
  uint8_t* img = smem + kMetaBytes;
  const TileView tile = make_tile(img + P.stage_bytes + 64, P.tile_items);
  const int lane = threadIdx.x;
  const uint32_t b_begin = blockIdx.x * P.blocks_per_wave;
  const uint32_t b_end = min(b_begin + P.blocks_per_wave, P.n_blocks);

  for (uint32_t b = b_begin; b < b_end;) {
    // ---- group formation: longest run b..b+k-1 fitting stage + tile
    const uint64_t off_b = P.block_off[b];
    const uint64_t span0 = off_b & ~15ULL;
    const uint32_t g_item0 = P.item_start[b];
    const uint32_t bj = b + lane;
    bool fits = false;
    if (bj < b_end) {
      const uint64_t hi = P.block_off[bj + 1];
      const uint64_t need = ((hi + 15) & ~15ULL) - span0;
      const uint32_t items = P.item_start[bj + 1] - g_item0;
      fits = hi >= off_b && need <= P.stage_bytes && items <= P.tile_items;
    }
    const uint64_t fit_mask = __ballot(fits);
    const uint32_t k = (fit_mask == ~0ULL) ? 64u : (uint32_t)__builtin_ctzll(~fit_mask);
    if (k == 0) {
      decode_block_direct(P, b, meta);
      b += 1;
      continue;
    }
    // ---- stage the run's bytes HBM -> LDS (16 B per lane per step)
    {
      const uint64_t span1 = (P.block_off[b + k] + 15) & ~15ULL;
      const uint32_t chunks = (uint32_t)((span1 - span0) >> 4);
      const u32x4* __restrict__ src = reinterpret_cast<const u32x4*>(P.blocks + span0);
      u32x4* dst = reinterpret_cast<u32x4*>(img);
      uint32_t c = lane;
      for (; c + 3 * kWave < chunks; c += 4 * kWave) {
        u32x4 v0 = __builtin_nontemporal_load(src + c);
        u32x4 v1 = __builtin_nontemporal_load(src + c + kWave);
        u32x4 v2 = __builtin_nontemporal_load(src + c + 2 * kWave);
        u32x4 v3 = __builtin_nontemporal_load(src + c + 3 * kWave);
        dst[c] = v0;
        dst[c + kWave] = v1;
        dst[c + 2 * kWave] = v2;
        dst[c + 3 * kWave] = v3;
      }
      for (; c < chunks; c += kWave) dst[c] = __builtin_nontemporal_load(src + c);
    }
    __syncthreads();
    // ---- lane j: header of block b+j
    if ((uint32_t)lane < k) {
      const uint64_t off = P.block_off[b + lane], end = P.block_off[b + lane + 1];
      BlockMeta m;
      meta_header(img, (uint32_t)(off - span0), end - off, m);
      m.item0 = P.item_start[b + lane] - g_item0;
      meta[lane] = m;
    }
    __syncthreads();
    // ---- payload checksums, one block at a time, whole wave
    for (uint32_t j = 0; j < k; ++j) {
      if (meta[j].st != ST_OK) continue;
      const uint32_t hb = meta[j].hb, len = meta[j].len;
      uint64_t lo, hi;
      xxh3_128_wave(img, hb + kHdrLen, len - kHdrLen, &kLongSecret, lo, hi);
      if (lane == 0 && (lo != meta[j].ck_lo || hi != meta[j].ck_hi)) meta[j].st = ST_CKSUM;
    }
    __syncthreads();
    // ---- trailers + interval prefix
    uint32_t chains = 0;
    if ((uint32_t)lane < k) {
      BlockMeta m = meta[lane];
      const uint32_t cap = P.item_start[b + lane + 1] - P.item_start[b + lane];
      meta_trailer(img, P.expect_type, cap, m);
      chains = m.st == ST_OK ? m.bin_len : 0;
      meta[lane] = m;
    }
    const uint32_t incl = wave_incl_scan_u32(chains);
    const uint32_t total = wave_bcast_u32(incl, 63);
    if ((uint32_t)lane < k) meta[lane].chain0 = incl - chains;
    __syncthreads();
    // ---- walk restart intervals: lane = (block, interval)
    for (uint32_t c = lane; c < total; c += kWave) {
      uint32_t lo = 0, hi = k - 1;
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (meta[mid].chain0 <= c) lo = mid; else hi = mid - 1;
      }
      const BlockMeta& mm = meta[lo];
      const uint32_t r = c - mm.chain0;
      const uint32_t item0 = mm.item0;
      bool ok;
      if (mm.type == 1 && P.out.handle_off) {
        const uint64_t gbase = (uint64_t)g_item0 + item0;
        ok = walk_interval(img, mm.hb + kHdrLen, mm, r, [&](uint32_t j, const ItemFields& f) {
          emit_tile(tile, item0 + j, f);
          P.out.handle_off[gbase + j] = f.handle_off;
        });
      } else {
        ok = walk_interval(img, mm.hb + kHdrLen, mm, r,
                           [&](uint32_t j, const ItemFields& f) { emit_tile(tile, item0 + j, f); });
      }
      if (!ok) atomicCAS(&meta[lo].st, ST_OK, ST_PARSE);
    }
    __syncthreads();
    // ---- data-block handle_off (documented as 0 for data items)
    if (P.out.handle_off) {
      for (uint32_t j = 0; j < k; ++j) {
        if (meta[j].type == 1) continue;
        const uint32_t n0 = meta[j].item0, n1 = j + 1 < k ? meta[j + 1].item0 : P.item_start[b + k] - g_item0;
        for (uint32_t i = n0 + lane; i < n1; i += kWave) P.out.handle_off[(uint64_t)g_item0 + i] = 0;
      }
    }
    // ---- tile -> HBM, coalesced per field
    {
      const uint32_t n = P.item_start[b + k] - g_item0;
      const uint64_t g0 = g_item0;
      if (P.out.seqno) for (uint32_t i = lane; i < n; i += kWave) P.out.seqno[g0 + i] = tile.seqno[i];
      if (P.out.key_off) for (uint32_t i = lane; i < n; i += kWave) P.out.key_off[g0 + i] = tile.key_off[i];
      if (P.out.val_off) for (uint32_t i = lane; i < n; i += kWave) P.out.val_off[g0 + i] = tile.val_off[i];
      if (P.out.val_len) for (uint32_t i = lane; i < n; i += kWave) P.out.val_len[g0 + i] = tile.val_len[i];
      if (P.out.key_len) for (uint32_t i = lane; i < n; i += kWave) P.out.key_len[g0 + i] = tile.key_len[i];
      if (P.out.prefix_len) for (uint32_t i = lane; i < n; i += kWave) P.out.prefix_len[g0 + i] = tile.prefix_len[i];
      if (P.out.vtype) for (uint32_t i = lane; i < n; i += kWave) P.out.vtype[g0 + i] = tile.vtype[i];
    }
    if ((uint32_t)lane < k) P.status[b + lane] = meta[lane].st;
    __syncthreads();
    b += k;
  }
}

// item counts from the trailers (trailer.rs:57-75), same rule as
// oracle/batch.c: 0 unless the handle holds header + a 32-byte minimum payload,
// and at most (payload - 32) / 3 (every record is >= 3 bytes), so a corrupt,
// not-yet-verified trailer cannot reserve more than its bytes could hold.
__global__ __launch_bounds__(256) void trailer_counts_kernel(const uint8_t* __restrict__ blocks,
                                                             const uint64_t* __restrict__ off, uint32_t n,
                                                             uint64_t* __restrict__ counts) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  const uint64_t o = off[b], e = off[b + 1];
  uint64_t c = 0;
  if (e >= o && e - o >= kHdrLen + kTrailerLen + 1) {
    const uint8_t* p = blocks + e - 4;
    c = (uint64_t)p[0] | ((uint64_t)p[1] << 8) | ((uint64_t)p[2] << 16) | ((uint64_t)p[3] << 24);
    const uint64_t most = (e - o - kHdrLen - 32) / 3;  // records are >= 3 bytes each
    c = c < most ? c : most;
  }
  counts[b] = c;
}

struct ItemStartOut {
  uint32_t* item_start;
  uint64_t cap;
  __device__ void operator()(uint64_t i, uint64_t prefix) const {
    item_start[i] = (uint32_t)(prefix < cap ? prefix : cap);
  }
};

size_t decode_workspace_size(uint32_t n_blocks) {
  return ((size_t)n_blocks * 8 + 255) / 256 * 256 + (scan_tiles(n_blocks) * 8 + 255) / 256 * 256;
}

uint32_t decode_lds_bytes(uint32_t stage_bytes, uint32_t tile_items) {
  return kMetaBytes + stage_bytes + 64 + tile_bytes(tile_items);
}

hipError_t launch_decode(const DecodeParams& P0, void* ws, hipStream_t st) {
  DecodeParams P = P0;
  uint64_t* counts = (uint64_t*)ws;
  uint64_t* tiles = (uint64_t*)((uint8_t*)ws + ((size_t)P.n_blocks * 8 + 255) / 256 * 256);
  if (!(P.flags & LSM_DECODE_ITEM_START_VALID)) {
    hipLaunchKernelGGL(trailer_counts_kernel, dim3((P.n_blocks + 255) / 256), dim3(256), 0, st, P.blocks,
                       P.block_off, P.n_blocks, counts);
    hipError_t e = launch_excl_scan(counts, P.n_blocks, tiles, ItemStartOut{P.item_start_w, P.item_cap}, st);
    if (e != hipSuccess) return e;
  }
  const uint32_t lds = decode_lds_bytes(P.stage_bytes, P.tile_items);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)decode_blocks_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  const uint32_t grid = (P.n_blocks + P.blocks_per_wave - 1) / P.blocks_per_wave;
  hipLaunchKernelGGL(decode_blocks_kernel, dim3(grid), dim3(64), lds, st, P);
  return hipGetLastError();
}

}  // namespace lsmgpu
