// point_read.hip — batched DataBlock::point_read and the
// range seeks of the data-block iterator (§8(a) a13) on gfx950.
//
// Replaces, per query, DataBlock::point_read(needle, seqno)
// (src/table/data_block/mod.rs:412-472) on an already-loaded block: the
// hash-index probe (hash_index/reader.rs:46-58, bucket =
// xxh3_64(needle) % buckets, hash_index/mod.rs:35-41), on FREE "not found",
// on CONFLICT or without a hash index the restart-head binary search
// (block/decoder.rs:153-207, iter.rs:37-76: start at the last restart head
// whose key is < needle, else at 0), else the head the bucket names; then
// the linear scan of data_block/mod.rs:447-469 with compare_prefixed_slice
// (src/table/util.rs:133-167): key > needle -> not found, key < needle ->
// next, key == needle and seqno >= snapshot -> next (MVCC), else found.
//
// One lane per query, straight from HBM: the block bytes are read through the
// same aligned-window Cursor the general decode path uses, keys are compared
// 16 bytes per step.  Blocks are taken as loaded by Block::from_file (the
// payload checksum was verified there): header fields and the trailer are
// checked structurally, the payload checksum is not re-computed.
#include <hip/hip_runtime.h>

#include "block_format.hpp"
#include "decode.hpp"
#include "lsmgpu.h"

namespace lsmgpu {

struct PointReadParams {
  const uint8_t* blocks;
  const uint64_t* block_off;
  uint32_t n_blocks;
  const uint32_t* q_block;
  const uint8_t* needles;
  const uint64_t* needle_off;
  const uint64_t* snapshot;
  uint32_t n;
  lsm_point_result out;
  int32_t* status;
};

__device__ __forceinline__ uint32_t win_byte(const Win16& w, uint32_t i) {
  return (uint32_t)((i < 8 ? w.lo >> (8 * i) : w.hi >> (8 * (i - 8))) & 0xFF);
}

// Lexicographic compare of a[ap .. ap+an) with b[bp .. bp+bn) (both bases
// 4-byte aligned, 16-byte windows; both spans readable up to 20 bytes past).
__device__ __forceinline__ int cmp_span(const uint8_t* ab, uint32_t ap, uint32_t an, const uint8_t* bb, uint32_t bp,
                                        uint32_t bn) {
  const uint32_t n = min(an, bn);
  for (uint32_t k = 0; k < n; k += 16) {
    const Win16 wa = read_win16(ab, ap + k), wb = read_win16(bb, bp + k);
    const uint32_t m = min(16u, n - k);
    uint64_t x0 = wa.lo ^ wb.lo, x1 = wa.hi ^ wb.hi;
    if (m < 8) {
      x0 &= (1ULL << (8 * m)) - 1;
      x1 = 0;
    } else if (m < 16) {
      x1 &= m == 8 ? 0ULL : (1ULL << (8 * (m - 8))) - 1;
    }
    if (x0 | x1) {
      const uint32_t i = x0 ? (uint32_t)__builtin_ctzll(x0) >> 3 : 8 + ((uint32_t)__builtin_ctzll(x1) >> 3);
      return win_byte(wa, i) < win_byte(wb, i) ? -1 : 1;
    }
  }
  return an < bn ? -1 : (an > bn ? 1 : 0);
}

// compare_prefixed_slice(prefix, suffix, needle), src/table/util.rs:133-167.
__device__ __forceinline__ int cmp_prefixed(const uint8_t* kb, uint32_t pre, uint32_t pn, uint32_t suf, uint32_t sn,
                                            const uint8_t* nb, uint32_t np, uint32_t nn) {
  if (nn == 0) return (pn + sn) > 0 ? 1 : 0;
  const uint32_t m = min(pn, nn);
  const int c = cmp_span(kb, pre, m, nb, np, m);
  if (c) return c;
  if (pn > nn) return 1;
  return cmp_span(kb, suf, sn, nb, np + pn, nn - pn);
}

__global__ __launch_bounds__(256) void point_read_kernel(PointReadParams P) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= P.n) return;
  int32_t st = ST_OK;
  int64_t found = -1;
  ItemFields hit{};
  const uint32_t b = P.q_block[q];
  if (b >= P.n_blocks) {
    P.status[q] = ST_BAD_ARG;
    P.out.item[q] = -1;
    return;
  }
  const uint64_t off = P.block_off[b], end = P.block_off[b + 1];
  const uint8_t* base = P.blocks + (off & ~15ULL);
  const uint32_t hb = (uint32_t)(off & 15);
  const uint64_t len = end >= off ? end - off : 0;
  const uint64_t no = P.needle_off[q];
  const uint32_t nn = (uint32_t)min(P.needle_off[q + 1] - no, (uint64_t)0xFFFFFFFFu);
  const uint8_t* nb = P.needles + (no & ~15ULL);
  const uint32_t np = (uint32_t)(no & 15);
  const uint64_t snap = P.snapshot[q];
  HeaderInfo h;
  st = check_header_fields(base, hb, len, h);
  if (st == ST_OK && h.data_length != len - kHdrLen) st = ST_TRUNCATED;
  if (st == ST_OK && h.type != LSM_BLOCK_DATA && h.type != LSM_BLOCK_META) st = ST_TYPE_MISMATCH;
  TrailerInfo t;
  const uint32_t p0 = hb + kHdrLen;
  if (st == ST_OK) st = read_trailer(base, p0, h.data_length, t);
  if (st == ST_OK) {
    bool search = true, miss = false;
    uint32_t start = 0;
    if (t.hash_len > 0) {
      if ((uint64_t)t.hash_off + t.hash_len > (uint64_t)h.data_length - kTrailerLen) {  // bucket bytes precede the trailer
        st = ST_PARSE;
      } else {
        const uint64_t hv = xxh3_64_any(nn, BaseReader8{nb, np}, BaseReader64{nb, np});
        const uint32_t m = read_u32_unaligned(base, p0 + t.hash_off + (uint32_t)(hv % t.hash_len)) & 0xFF;
        if (m == kHashFree) {
          miss = true;
        } else if (m != kHashConflict) {
          if (m >= t.bin_len) st = ST_PARSE;
          start = m;
          search = false;
        }
      }
    }
    if (st == ST_OK && !miss && search) {  // last restart head with key < needle
      uint32_t lo = 0, hi = t.bin_len;
      while (lo < hi && st == ST_OK) {
        const uint32_t mid = lo + (hi - lo) / 2;
        Cursor c;
        c.init(base, p0, bin_get(base, p0, t, mid), t.rec_end);
        ItemFields f;
        if (!parse_data_record(c, true, 0, f)) {
          st = ST_PARSE;
          break;
        }
        if (cmp_span(base, p0 + f.key_off, f.key_len, nb, np, nn) < 0) lo = mid + 1;
        else hi = mid;
      }
      start = lo == 0 ? 0 : lo - 1;
    }
    if (st == ST_OK && !miss) {  // linear scan from restart head `start`
      Cursor c;
      c.init(base, p0, bin_get(base, p0, t, start), t.rec_end);
      uint32_t head_key = 0;
      for (uint64_t i = (uint64_t)start * t.ri; i < t.item_count; ++i) {
        const bool restart = i % t.ri == 0;
        ItemFields f;
        if (!parse_data_record(c, restart, head_key, f)) {
          st = ST_PARSE;
          break;
        }
        int cmp;
        if (restart) {
          head_key = f.key_off;
          cmp = cmp_span(base, p0 + f.key_off, f.key_len, nb, np, nn);
        } else {
          cmp = cmp_prefixed(base, p0 + head_key, f.prefix_len, p0 + f.key_off, f.key_len, nb, np, nn);
        }
        if (cmp > 0) break;
        if (cmp < 0) continue;
        if (f.seqno >= snap) continue;
        found = (int64_t)i;
        hit = f;
        break;
      }
    }
  }
  P.status[q] = st;
  P.out.item[q] = st == ST_OK ? (int32_t)found : -1;
  if (found >= 0) {
    if (P.out.seqno) P.out.seqno[q] = hit.seqno;
    if (P.out.val_off) P.out.val_off[q] = hit.val_off;
    if (P.out.val_len) P.out.val_len[q] = hit.val_len;
    if (P.out.vtype) P.out.vtype[q] = hit.vtype;
  }
}

// ---------------------------------------------------------------- seek
// Batched Iter::seek / seek_exclusive / seek_upper / seek_upper_exclusive
// (src/table/data_block/iter.rs:37-176) on an already-loaded data block: the
// item range [first, end) that next() / next_back() / any ping-pong of them
// yield after the given bounds, and the seeks' return values.  Lane per query.
// Each bound is Decoder::partition_point over the restart heads
// (block/decoder.rs:153-207: the last head with key < needle (lower bound) or
// key <= needle (upper bound), else head 0) plus a linear scan with
// compare_prefixed_slice.  The reference scans the upper bound backwards from
// the end of its interval; on a sorted block the forward scan used here stops
// at the same item (the first key > needle, or >= needle when exclusive).
struct SeekParams {
  const uint8_t* blocks;
  const uint64_t* block_off;
  uint32_t n_blocks;
  const uint32_t* q_block;
  const uint8_t* lo;
  const uint64_t* lo_off;
  const uint8_t* hi;
  const uint64_t* hi_off;
  const uint8_t* flags;
  uint32_t n;
  uint32_t* first;
  uint32_t* end;
  uint8_t* found;
  int32_t* status;
};

// partition_point over the restart heads: pred = head < needle (or <= with le).
__device__ __forceinline__ int32_t seek_partition(const uint8_t* base, uint32_t p0, const TrailerInfo& t,
                                                  const uint8_t* nb, uint32_t np, uint32_t nn, bool le,
                                                  uint32_t& iv) {
  uint32_t lo = 0, hi = t.bin_len;
  while (lo < hi) {
    const uint32_t mid = lo + (hi - lo) / 2;
    Cursor c;
    c.init(base, p0, bin_get(base, p0, t, mid), t.rec_end);
    ItemFields f;
    if (!parse_data_record(c, true, 0, f)) return ST_PARSE;
    const int cmp = cmp_span(base, p0 + f.key_off, f.key_len, nb, np, nn);
    if (le ? cmp <= 0 : cmp < 0) lo = mid + 1;
    else hi = mid;
  }
  iv = lo == 0 ? 0 : lo - 1;
  return ST_OK;
}

// Forward scan from restart interval iv: index of the first item that stops
// it (key >= needle, or key > needle with `past_equal`), item_count if none;
// eq = that item's key equals the needle.
__device__ __forceinline__ int32_t seek_scan(const uint8_t* base, uint32_t p0, const TrailerInfo& t, uint32_t iv,
                                             const uint8_t* nb, uint32_t np, uint32_t nn, bool past_equal,
                                             uint32_t& at, bool& eq, bool& prev_eq) {
  Cursor c;
  c.init(base, p0, bin_get(base, p0, t, iv), t.rec_end);
  uint32_t head_key = 0;
  at = t.item_count;
  eq = prev_eq = false;
  for (uint32_t i = iv * t.ri; i < t.item_count; ++i) {
    const bool restart = i % t.ri == 0;
    ItemFields f;
    if (!parse_data_record(c, restart, head_key, f)) return ST_PARSE;
    int cmp;
    if (restart) {
      head_key = f.key_off;
      cmp = cmp_span(base, p0 + f.key_off, f.key_len, nb, np, nn);
    } else {
      cmp = cmp_prefixed(base, p0 + head_key, f.prefix_len, p0 + f.key_off, f.key_len, nb, np, nn);
    }
    if (cmp > 0 || (cmp == 0 && !past_equal)) {
      at = i;
      eq = cmp == 0;
      return ST_OK;
    }
    prev_eq = cmp == 0;
  }
  return ST_OK;
}

__global__ __launch_bounds__(256) void seek_kernel(SeekParams P) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= P.n) return;
  const uint32_t b = P.q_block[q];
  const uint32_t fl = P.flags[q];
  int32_t st = ST_OK;
  uint32_t first = 0, end = 0, found = 0;
  if (b >= P.n_blocks) st = ST_BAD_ARG;
  const uint64_t off = st == ST_OK ? P.block_off[b] : 0, bend = st == ST_OK ? P.block_off[b + 1] : 0;
  const uint8_t* base = P.blocks + (off & ~15ULL);
  const uint32_t hb = (uint32_t)(off & 15);
  const uint64_t len = bend >= off ? bend - off : 0;
  HeaderInfo h;
  TrailerInfo t;
  const uint32_t p0 = hb + kHdrLen;
  if (st == ST_OK) st = check_header_fields(base, hb, len, h);
  if (st == ST_OK && h.data_length != len - kHdrLen) st = ST_TRUNCATED;
  if (st == ST_OK && h.type != LSM_BLOCK_DATA && h.type != LSM_BLOCK_META) st = ST_TYPE_MISMATCH;
  if (st == ST_OK) st = read_trailer(base, p0, h.data_length, t);
  if (st == ST_OK) {
    first = 0;
    end = t.item_count;
    if (fl & LSM_SEEK_LO) {  // Iter::seek (iter.rs:37-76) / seek_exclusive (iter.rs:115-145)
      const uint64_t o = P.lo_off[q];
      const uint32_t nn = (uint32_t)min(P.lo_off[q + 1] - o, (uint64_t)0xFFFFFFFFu);
      const uint8_t* nb = P.lo + (o & ~15ULL);
      const uint32_t np = (uint32_t)(o & 15);
      const bool excl = (fl & LSM_SEEK_LO_EXCLUSIVE) != 0;
      uint32_t iv = 0;
      bool eq = false, prev_eq = false;
      st = seek_partition(base, p0, t, nb, np, nn, false, iv);
      if (st == ST_OK) st = seek_scan(base, p0, t, iv, nb, np, nn, excl, first, eq, prev_eq);
      if (excl ? first < t.item_count : eq) found |= 1;
    }
    if (st == ST_OK && (fl & LSM_SEEK_HI)) {  // Iter::seek_upper (iter.rs:78-113) / seek_upper_exclusive (:147-176)
      const uint64_t o = P.hi_off[q];
      const uint32_t nn = (uint32_t)min(P.hi_off[q + 1] - o, (uint64_t)0xFFFFFFFFu);
      const uint8_t* nb = P.hi + (o & ~15ULL);
      const uint32_t np = (uint32_t)(o & 15);
      const bool excl = (fl & LSM_SEEK_HI_EXCLUSIVE) != 0;
      uint32_t iv = 0;
      bool eq = false, prev_eq = false;
      // inclusive: end = first key > needle (heads <= needle); exclusive: first key >= needle (heads < needle)
      st = seek_partition(base, p0, t, nb, np, nn, !excl, iv);
      if (st == ST_OK) st = seek_scan(base, p0, t, iv, nb, np, nn, !excl, end, eq, prev_eq);
      if (excl ? end > 0 : (end > 0 && prev_eq)) found |= 2;
    }
    if (first > end) first = end;  // the two scanners crossed: empty range
  }
  P.status[q] = st;
  P.first[q] = st == ST_OK ? first : 0;
  P.end[q] = st == ST_OK ? end : 0;
  if (P.found) P.found[q] = (uint8_t)(st == ST_OK ? found : 0);
}

hipError_t launch_point_read(const uint8_t* blocks, const uint64_t* block_off, uint32_t n_blocks, const uint32_t* q_block,
                             const uint8_t* needles, const uint64_t* needle_off, const uint64_t* snapshot, uint32_t n,
                             const lsm_point_result& out, int32_t* status, hipStream_t st) {
  PointReadParams P{blocks, block_off, n_blocks, q_block, needles, needle_off, snapshot, n, out, status};
  hipLaunchKernelGGL(point_read_kernel, dim3((n + 255) / 256), dim3(256), 0, st, P);
  return hipGetLastError();
}

hipError_t launch_seek(const SeekParams& P, hipStream_t st) {
  hipLaunchKernelGGL(seek_kernel, dim3((P.n + 255) / 256), dim3(256), 0, st, P);
  return hipGetLastError();
}

}  // namespace lsmgpu

extern "C" int lsm_seek_blocks(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                               const uint32_t* d_query_block, const uint8_t* d_lo, const uint64_t* d_lo_off,
                               const uint8_t* d_hi, const uint64_t* d_hi_off, const uint8_t* d_flags,
                               uint32_t n_queries, uint32_t* d_first, uint32_t* d_end, uint8_t* d_found,
                               int32_t* d_status, void* stream) {
  if (n_queries == 0) return LSM_OK;
  if (!d_blocks || !d_block_off || !d_query_block || !d_flags || !d_first || !d_end || !d_status) return LSM_BAD_ARG;
  if (!d_lo || !d_lo_off || !d_hi || !d_hi_off) return LSM_BAD_ARG;
  if (((uintptr_t)d_blocks & 15) || ((uintptr_t)d_lo & 15) || ((uintptr_t)d_hi & 15)) return LSM_BAD_ARG;
  lsmgpu::SeekParams P{d_blocks, d_block_off, n_blocks, d_query_block, d_lo, d_lo_off, d_hi, d_hi_off, d_flags,
                       n_queries, d_first, d_end, d_found, d_status};
  return lsmgpu::hip_status(lsmgpu::launch_seek(P, (hipStream_t)stream), "lsm_seek_blocks");
}

extern "C" int lsm_point_read_blocks(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                                     const uint32_t* d_query_block, const uint8_t* d_needles,
                                     const uint64_t* d_needle_off, const uint64_t* d_snapshot, uint32_t n_queries,
                                     const lsm_point_result* d_out, int32_t* d_status, void* stream) {
  if (n_queries == 0) return LSM_OK;
  if (!d_blocks || !d_block_off || !d_query_block || !d_needles || !d_needle_off || !d_snapshot || !d_out ||
      !d_out->item || !d_status)
    return LSM_BAD_ARG;
  // the kernel reads blocks and needles through aligned 4-byte windows from 16-byte-aligned bases
  if (((uintptr_t)d_blocks & 15) || ((uintptr_t)d_needles & 15)) return LSM_BAD_ARG;
  const hipError_t e = lsmgpu::launch_point_read(d_blocks, d_block_off, n_blocks, d_query_block, d_needles,
                                                 d_needle_off, d_snapshot, n_queries, *d_out, d_status,
                                                 (hipStream_t)stream);
  return lsmgpu::hip_status(e, "lsm_point_read_blocks");
}
