// table_scan.hip — whole-table scan: Scanner::new / next
// (src/table/scanner.rs:24-92) over a table file image in HBM.
//
// Scanner reads the data blocks back to back from file offset 0 with
// Block::from_reader, so each block's position depends on the previous
// header: a serial chain.  On the device the positions come from the table's
// block index instead, which the writer records for every data block
// (KeyedBlockHandle(last key, seqno, (file_pos, 33 + data_length)),
// writer/mod.rs:328-335):
//   level 1  the TLI block (the TOC "tli" section, regions.rs:55-76) is an
//            index block; with a full index its entries are the data blocks
//            (writer/index/full.rs:55-69), with a two-level index they are the
//            index partitions (writer/index/partitioned.rs:54-125, offsets
//            already shifted to the file, :136-140);
//   level 2  (two-level only) the partitions are decoded as one batch;
//   data     handles -> block offsets (contiguity checked), then one
//            lsm_decode_blocks pass over every data block with the table's
//            global_seqno added to each item (scanner.rs:84).
// Index levels are decoded by the same decode kernels (index blocks take the
// general path).  lsm_scan_table reads each level's entry count back to size
// the next launch (one stream synchronisation per index level);
// lsm_scan_table_async keeps the counts on the device and launches each level
// for the caller's bounds.
#include <hip/hip_runtime.h>
#include "fill.hpp"

#include "decode.hpp"
#include "lsmgpu.h"

namespace lsmgpu {

// Handles of one index level -> block offsets for lsm_decode_blocks (n+1
// entries).  bad[0] = the first entry whose handle does not start where the
// previous one ended (or, for the data level, the first block not at 0),
// runs past the file or is shorter than a header; 0xFFFFFFFF if none.
__global__ __launch_bounds__(256) void handles_to_offsets_kernel(const uint64_t* __restrict__ h_off,
                                                                 const uint32_t* __restrict__ h_size, uint32_t n,
                                                                 uint64_t file_len, uint64_t first_at,
                                                                 uint64_t* __restrict__ block_off,
                                                                 uint32_t* __restrict__ bad) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint64_t o = h_off[i], sz = h_size[i];
  const uint64_t e = o + sz;
  bool ok = sz >= 33 && e >= o && e <= file_len;
  if (i == 0) ok = ok && (first_at == ~0ULL || o == first_at);
  if (i + 1 < n) ok = ok && h_off[i + 1] == e;
  block_off[i] = o;
  if (i + 1 == n) block_off[n] = e;
  if (!ok) atomicMin(bad, i);
}

// First failing block of a level: bad[0] = min index with status != OK.
__global__ __launch_bounds__(256) void first_failed_kernel(const int32_t* __restrict__ status, uint32_t n,
                                                           uint32_t* __restrict__ bad) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n && status[i] != LSM_OK) atomicMin(bad, i);
}

__global__ void tli_handle_kernel(uint64_t* block_off, uint64_t off, uint64_t end) {
  block_off[0] = off;
  block_off[1] = end;
}

// ---- lsm_scan_table_async: the same walk with every count kept on the device.
// Each level is launched for the caller's bound (cap + 1 index blocks, the data
// blocks' hint); the blocks past a level's real count are empty ranges (their
// statuses are not looked at), and a failed level empties every later range,
// so nothing after it reads or writes anything but empty blocks.
struct ScanState {
  uint32_t n_lvl;         // entries of the level being decoded
  int32_t table_status;   // LSM_OK until a level fails
  uint32_t dead;          // a level failed: later ranges are empty
  uint32_t pad;
};

// One workgroup after an index level's decode: its first failing block, its
// entry count, the bounds (at most cap, at least one; the data level's count
// equals block_count when that is non-zero).
__global__ __launch_bounds__(256) void scan_level_check_kernel(ScanState* st, const int32_t* __restrict__ status,
                                                               const uint32_t* __restrict__ item_start, uint32_t cap,
                                                               uint32_t block_count, uint32_t data_level) {
  __shared__ uint32_t first;
  if (threadIdx.x == 0) first = 0xFFFFFFFFu;
  __syncthreads();
  const uint32_t n = st->n_lvl;
  const bool dead = st->dead != 0;
  for (uint32_t i = threadIdx.x; !dead && i < n; i += 256)
    if (status[i] != LSM_OK) atomicMin(&first, i);
  __syncthreads();
  if (threadIdx.x != 0 || dead) return;
  int32_t ts = LSM_OK;
  const uint32_t entries = item_start[n];
  if (first != 0xFFFFFFFFu) ts = status[first];
  else if (entries > cap) ts = LSM_OVERFLOW;
  else if (entries == 0) ts = LSM_PARSE;  // (the writer never leaves an index empty)
  else if (data_level && block_count && block_count != entries) ts = LSM_PARSE;
  if (ts != LSM_OK) {
    st->table_status = ts;
    st->dead = 1;
  } else {
    st->n_lvl = entries;
  }
}

// Handles -> offsets [0, last]: entries as handles_to_offsets_kernel,
// the rest empty at the last end; a dead scan leaves every range empty at 0.
__global__ __launch_bounds__(256) void scan_handles_kernel(const ScanState* st, const uint64_t* __restrict__ h_off,
                                                           const uint32_t* __restrict__ h_size, uint32_t last,
                                                           uint64_t file_len, uint64_t first_at,
                                                           uint64_t* __restrict__ block_off, uint32_t* __restrict__ bad) {
  const uint32_t n = st->n_lvl;
  const bool dead = st->dead != 0;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i <= last; i += gridDim.x * 256) {
    if (dead) {
      block_off[i] = 0;
      continue;
    }
    if (i >= n) {  // past the level: empty ranges at its end
      block_off[i] = h_off[n - 1] + h_size[n - 1];
      continue;
    }
    const uint64_t o = h_off[i], sz = h_size[i];
    const uint64_t e = o + sz;
    bool ok = sz >= 33 && e >= o && e <= file_len;
    if (i == 0) ok = ok && (first_at == ~0ULL || o == first_at);
    if (i + 1 < n) ok = ok && h_off[i + 1] == e;
    block_off[i] = o;
    if (!ok) atomicMin(bad, i);
  }
}

// A handle check failed: TRUNCATED, every range emptied.
__global__ __launch_bounds__(256) void scan_handles_fail_kernel(ScanState* st, const uint32_t* __restrict__ bad,
                                                                uint32_t last, uint64_t* __restrict__ block_off) {
  const bool skip = bad[0] == 0xFFFFFFFFu || st->dead;
  __syncthreads();  // (every thread has read st before thread 0 changes it)
  if (skip) return;
  for (uint32_t i = threadIdx.x; i <= last; i += 256) block_off[i] = 0;
  if (threadIdx.x == 0) {
    st->table_status = LSM_TRUNCATED;
    st->dead = 1;
  }
}

__global__ void scan_result_kernel(const ScanState* st, uint32_t* n_blocks, int32_t* table_status) {
  *n_blocks = st->dead ? 0u : st->n_lvl;
  *table_status = st->table_status;
}

}  // namespace lsmgpu

using namespace lsmgpu;

namespace {

constexpr size_t align256(size_t x) { return (x + 255) / 256 * 256; }

// Workspace carve (every level holds at most cap + 1 entries / blocks).
struct ScanWs {
  uint64_t* h_off;      // index entries: BlockHandle offsets
  uint32_t* h_size;     // index entries: BlockHandle sizes (parsed val_len)
  uint64_t* lvl_off;    // block offsets of the index level being decoded
  uint32_t* lvl_start;  // its item starts
  int32_t* lvl_status;  // its statuses
  uint32_t* flag;       // [0] first bad entry, [1] first failed block
  ScanState* state;     // lsm_scan_table_async
  void* dec_ws;
  size_t dec_bytes;
};

size_t scan_ws_size(uint32_t cap, ScanWs* w, uint8_t* base) {
  const size_t e = (size_t)cap + 1;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    uint8_t* p = base ? base + o : nullptr;
    o += align256(bytes);
    return p;
  };
  ScanWs tmp;
  ScanWs& s = w ? *w : tmp;
  s.h_off = (uint64_t*)take(8 * e);
  s.h_size = (uint32_t*)take(4 * e);
  s.lvl_off = (uint64_t*)take(8 * (e + 1));
  s.lvl_start = (uint32_t*)take(4 * (e + 1));
  s.lvl_status = (int32_t*)take(4 * e);
  s.flag = (uint32_t*)take(16);
  s.state = (ScanState*)take(sizeof(ScanState));
  s.dec_bytes = decode_workspace_size((uint32_t)e);
  s.dec_ws = take(s.dec_bytes);
  return o;
}

struct Sync {
  hipStream_t st;
  hipError_t e = hipSuccess;
  template <class T>
  T read(const T* d) {
    T v{};
    if (e == hipSuccess) e = hipMemcpyAsync(&v, d, sizeof(T), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    return v;
  }
};

DecodeParams index_params(const uint8_t* file, const uint64_t* off, uint32_t n, const ScanWs& w, uint32_t cap) {
  DecodeParams P{};
  P.blocks = file;
  P.block_off = off;
  P.n_blocks = n;
  P.expect_type = LSM_BLOCK_INDEX;
  P.out.handle_off = w.h_off;
  P.out.val_len = w.h_size;  // index blocks: val_len = BlockHandle size
  P.item_cap = cap;
  P.item_start = P.item_start_w = w.lvl_start;
  P.status = w.lvl_status;
  P.blocks_per_wave = kDefaultBlocksPerWave;
  P.stage_bytes = kDefaultStageBytes;
  P.tile_items = kDefaultTileItems;
  P.flags = 0;
  P.seqno_add = 0;
  return P;
}

}  // namespace

extern "C" size_t lsm_scan_workspace_size(uint32_t cap_blocks) { return scan_ws_size(cap_blocks, nullptr, nullptr); }

extern "C" int lsm_scan_table(const uint8_t* d_file, uint64_t file_len, const lsm_table_scan* table,
                              uint64_t* d_block_off, uint32_t cap_blocks, const lsm_parsed_items* d_out,
                              uint64_t item_cap, uint32_t* d_item_start, int32_t* d_status, uint32_t* n_blocks,
                              int32_t* table_status, void* d_workspace, size_t workspace_bytes, void* stream) {
  if (!d_file || !table || !d_block_off || !d_out || !d_item_start || !d_status || !n_blocks || !table_status ||
      !d_workspace || ((uintptr_t)d_file & 15) || cap_blocks == 0 || cap_blocks >= 0xFFFFFFF0u ||
      table->two_level > 1 || workspace_bytes < lsm_scan_workspace_size(cap_blocks))
    return LSM_BAD_ARG;
  *n_blocks = 0;
  *table_status = LSM_OK;
  const hipStream_t st = (hipStream_t)stream;
  ScanWs w;
  scan_ws_size(cap_blocks, &w, (uint8_t*)d_workspace);
  Sync sy{st};
  auto fail = [&](hipError_t e) { return hip_status(e, "lsm_scan_table"); };
  if (table->tli_size < 33 || table->tli_off + table->tli_size > file_len || table->tli_off + table->tli_size < table->tli_off) {
    *table_status = LSM_TRUNCATED;
    return LSM_OK;
  }
  // level 1: the TLI block
  hipLaunchKernelGGL(tli_handle_kernel, dim3(1), dim3(1), 0, st, w.lvl_off, table->tli_off,
                     table->tli_off + table->tli_size);
  uint32_t n_lvl = 1;
  const uint32_t levels = 1 + table->two_level;
  for (uint32_t lvl = 0; lvl < levels; ++lvl) {
    DecodeParams P = index_params(d_file, w.lvl_off, n_lvl, w, cap_blocks + 1);
    hipError_t e = launch_decode(P, w.dec_ws, w.dec_bytes, st);
    if (e == hipSuccess) e = fill_words_async(w.flag, 4, 0xFFFFFFFFu, st);
    if (e != hipSuccess) return fail(e);
    hipLaunchKernelGGL(first_failed_kernel, dim3((n_lvl + 255) / 256), dim3(256), 0, st, w.lvl_status, n_lvl,
                       w.flag + 1);
    const uint32_t bad = sy.read(w.flag + 1);
    const uint32_t entries = sy.read(w.lvl_start + n_lvl);
    if (sy.e != hipSuccess) return fail(sy.e);
    if (bad != 0xFFFFFFFFu) {
      *table_status = sy.read(w.lvl_status + bad);
      return sy.e == hipSuccess ? LSM_OK : fail(sy.e);
    }
    if (entries > cap_blocks) {
      *table_status = LSM_OVERFLOW;
      return LSM_OK;
    }
    if (entries == 0) {  // the writer never leaves an index empty (full.rs:85, partitioned.rs:226)
      *table_status = LSM_PARSE;
      return LSM_OK;
    }
    const bool data_level = lvl + 1 == levels;
    uint64_t* dst = data_level ? d_block_off : w.lvl_off;
    hipLaunchKernelGGL(handles_to_offsets_kernel, dim3((entries + 255) / 256), dim3(256), 0, st, w.h_off, w.h_size,
                       entries, file_len, data_level ? 0ULL : ~0ULL, dst, w.flag);
    const uint32_t hbad = sy.read(w.flag);
    if (sy.e != hipSuccess) return fail(sy.e);
    if (hbad != 0xFFFFFFFFu) {
      *table_status = LSM_TRUNCATED;
      return LSM_OK;
    }
    n_lvl = entries;
  }
  if (table->block_count && table->block_count != n_lvl) {
    *table_status = LSM_PARSE;
    return LSM_OK;
  }
  *n_blocks = n_lvl;
  // the data blocks: one decode pass, global_seqno added to every item
  DecodeParams P{};
  P.blocks = d_file;
  P.block_off = d_block_off;
  P.n_blocks = n_lvl;
  P.expect_type = LSM_BLOCK_DATA;
  P.out = *d_out;
  P.item_cap = item_cap > 0xFFFFFFFFULL ? 0xFFFFFFFFULL : item_cap;
  P.item_start = P.item_start_w = d_item_start;
  P.status = d_status;
  P.blocks_per_wave = kDefaultBlocksPerWave;
  P.stage_bytes = kDefaultStageBytes;
  P.tile_items = kDefaultTileItems;
  P.flags = 0;
  P.seqno_add = table->global_seqno;
  hipError_t e = launch_decode(P, w.dec_ws, w.dec_bytes, st);
  return e == hipSuccess ? LSM_OK : fail(e);
}

// The Scanner walk without host synchronisation (see lsm_scan_table_async in lsmgpu.h).
extern "C" int lsm_scan_table_async(const uint8_t* d_file, uint64_t file_len, const lsm_table_scan* table,
                                    uint64_t* d_block_off, uint32_t cap_blocks, uint32_t index_blocks_hint,
                                    uint32_t data_blocks_hint, const lsm_parsed_items* d_out, uint64_t item_cap, uint32_t* d_item_start,
                                    int32_t* d_status, uint32_t* d_n_blocks, int32_t* d_table_status,
                                    void* d_workspace, size_t workspace_bytes, void* stream) {
  if (!d_file || !table || !d_block_off || !d_out || !d_item_start || !d_status || !d_n_blocks || !d_table_status ||
      !d_workspace || ((uintptr_t)d_file & 15) || cap_blocks == 0 || cap_blocks >= 0xFFFFFFF0u ||
      table->two_level > 1 || workspace_bytes < lsm_scan_workspace_size(cap_blocks) || data_blocks_hint > cap_blocks ||
      index_blocks_hint > cap_blocks)
    return LSM_BAD_ARG;
  const uint32_t icap = index_blocks_hint ? index_blocks_hint : cap_blocks;  // the partition level's bound
  const hipStream_t st = (hipStream_t)stream;
  ScanWs w;
  scan_ws_size(cap_blocks, &w, (uint8_t*)d_workspace);
  auto fail = [&](hipError_t e) { return hip_status(e, "lsm_scan_table_async"); };
  const bool tli_ok = table->tli_size >= 33 && table->tli_off + table->tli_size <= file_len &&
                      table->tli_off + table->tli_size >= table->tli_off;
  ScanState s0{1, tli_ok ? (int32_t)LSM_OK : (int32_t)LSM_TRUNCATED, tli_ok ? 0u : 1u, 0};
  hipError_t e = hipMemcpyAsync(w.state, &s0, sizeof(s0), hipMemcpyHostToDevice, st);
  if (e != hipSuccess) return fail(e);
  hipLaunchKernelGGL(tli_handle_kernel, dim3(1), dim3(1), 0, st, w.lvl_off, tli_ok ? table->tli_off : 0,
                     tli_ok ? table->tli_off + table->tli_size : 0);
  const uint32_t levels = 1 + table->two_level;
  const uint32_t hgrid = min((cap_blocks + 256) / 256, 4096u);
  for (uint32_t lvl = 0; lvl < levels; ++lvl) {
    const uint32_t n_host = lvl == 0 ? 1 : icap;  // (bound on the level's blocks)
    DecodeParams P = index_params(d_file, w.lvl_off, n_host, w, cap_blocks + 1);
    if ((e = launch_decode(P, w.dec_ws, w.dec_bytes, st)) != hipSuccess) return fail(e);
    const bool data_level = lvl + 1 == levels;
    // (a level's entries must fit the next decode's ranges: the hints, else the cap)
    const uint32_t lvl_cap = data_level ? (data_blocks_hint ? data_blocks_hint : cap_blocks) : icap;
    hipLaunchKernelGGL(scan_level_check_kernel, dim3(1), dim3(256), 0, st, w.state, w.lvl_status, w.lvl_start,
                       lvl_cap, table->block_count, data_level ? 1u : 0u);
    if ((e = fill_words_async(w.flag, 4, 0xFFFFFFFFu, st)) != hipSuccess) return fail(e);
    uint64_t* dst = data_level ? d_block_off : w.lvl_off;
    // ranges [0, last]: the data decode reads up to cap + 1 offsets, the partition level icap + 1
    const uint32_t last = data_level ? cap_blocks : icap;
    hipLaunchKernelGGL(scan_handles_kernel, dim3(hgrid), dim3(256), 0, st, w.state, w.h_off, w.h_size, last,
                       file_len, data_level ? 0ULL : ~0ULL, dst, w.flag);
    hipLaunchKernelGGL(scan_handles_fail_kernel, dim3(1), dim3(256), 0, st, w.state, w.flag, last, dst);
  }
  hipLaunchKernelGGL(scan_result_kernel, dim3(1), dim3(1), 0, st, w.state, d_n_blocks, d_table_status);
  // the data blocks: the hint (or the cap) ranges, those past the real count empty
  DecodeParams P{};
  P.blocks = d_file;
  P.block_off = d_block_off;
  P.n_blocks = data_blocks_hint ? data_blocks_hint : cap_blocks;
  P.expect_type = LSM_BLOCK_DATA;
  P.out = *d_out;
  P.item_cap = item_cap > 0xFFFFFFFFULL ? 0xFFFFFFFFULL : item_cap;
  P.item_start = P.item_start_w = d_item_start;
  P.status = d_status;
  P.blocks_per_wave = kDefaultBlocksPerWave;
  P.stage_bytes = kDefaultStageBytes;
  P.tile_items = kDefaultTileItems;
  P.flags = 0;
  P.seqno_add = table->global_seqno;
  e = launch_decode(P, w.dec_ws, w.dec_bytes, st);
  return e == hipSuccess ? LSM_OK : fail(e);
}
