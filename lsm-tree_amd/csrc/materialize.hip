// materialize.hip — DataBlockParsedItem::materialize on the device
// (src/table/data_block/mod.rs:296-315): the owned key of every parsed item,
// Slice::fused(prefix, suffix) (src/slice/slice_default/mod.rs:44-46), where
// prefix = the first prefix_len bytes of the restart head's key and suffix =
// the item's own key bytes.  Values stay sub-slices of the block (val_off /
// val_len), as in the reference, so only keys are copied.
//   1. key_lengths_kernel  wave per block: len = prefix_len + key_len per item
//                          (0 for the items of a block whose status is not OK)
//   2. exclusive scan      -> d_key_out_off
//   3. materialize_kernel  wave per block, lane per item: the prefix from the
//                          head key (head = item - item % restart_interval,
//                          decoder.rs:442-483) then the suffix, byte stores.
#include <hip/hip_runtime.h>

#include "block_format.hpp"
#include "decode.hpp"
#include "lsmgpu.h"
#include "scan.hpp"

namespace lsmgpu {

struct MatParams {
  const uint8_t* blocks;
  const uint64_t* block_off;
  uint32_t n_blocks;
  const uint32_t* item_start;
  const int32_t* status;
  const uint32_t* key_off;
  const uint16_t* key_len;
  const uint16_t* prefix_len;
  uint64_t n_items;
  uint64_t* lens;
  uint8_t* out;
  const uint64_t* out_off;
};

// Restart interval of an OK block (trailer byte 0, trailer.rs:78-173).
__device__ __forceinline__ uint32_t block_restart_interval(const MatParams& P, uint32_t b) {
  const uint64_t e = P.block_off[b + 1];
  return P.blocks[e - kTrailerLen];
}

__global__ __launch_bounds__(256) void key_lengths_kernel(MatParams P) {
  const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= P.n_blocks) return;
  const uint64_t s = P.item_start[b], e = min((uint64_t)P.item_start[b + 1], P.n_items);
  const bool ok = P.status[b] == LSM_OK;
  for (uint64_t i = s + lane; i < e; i += 64) P.lens[i] = ok ? (uint64_t)P.prefix_len[i] + P.key_len[i] : 0;
}

__global__ __launch_bounds__(256) void materialize_kernel(MatParams P) {
  const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= P.n_blocks || P.status[b] != LSM_OK) return;
  const uint64_t s = P.item_start[b], e = min((uint64_t)P.item_start[b + 1], P.n_items);
  const uint8_t* payload = P.blocks + P.block_off[b] + kHdrLen;
  const uint32_t ri = block_restart_interval(P, b);
  for (uint64_t i = s + lane; i < e; i += 64) {
    const uint32_t k = (uint32_t)(i - s);
    const uint64_t head = s + (ri ? k - k % ri : k);
    const uint32_t pl = P.prefix_len[i], kl = P.key_len[i];
    uint8_t* dst = P.out + P.out_off[i];
    const uint8_t* pre = payload + P.key_off[head];
    const uint8_t* suf = payload + P.key_off[i];
    for (uint32_t j = 0; j < pl; ++j) dst[j] = pre[j];
    for (uint32_t j = 0; j < kl; ++j) dst[pl + j] = suf[j];
  }
}

struct KeyOffOut {
  uint64_t* off;
  __device__ void operator()(uint64_t i, uint64_t prefix) const { off[i] = prefix; }
};

}  // namespace lsmgpu

using namespace lsmgpu;

extern "C" size_t lsm_materialize_workspace_size(uint64_t n_items) {
  const uint64_t n = n_items ? n_items : 1;
  return (n * 8 + 255) / 256 * 256 + (scan_tiles(n) * 8 + 255) / 256 * 256;
}

static int mat_params(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                      const uint32_t* d_item_start, const int32_t* d_status, const lsm_parsed_items* d_parsed,
                      uint64_t n_items, uint64_t* d_key_out_off, MatParams& P) {
  if (!d_blocks || !d_block_off || !d_item_start || !d_status || !d_parsed || !d_parsed->key_off ||
      !d_parsed->key_len || !d_parsed->prefix_len || !d_key_out_off)
    return LSM_BAD_ARG;
  P.blocks = d_blocks;
  P.block_off = d_block_off;
  P.n_blocks = n_blocks;
  P.item_start = d_item_start;
  P.status = d_status;
  P.key_off = d_parsed->key_off;
  P.key_len = d_parsed->key_len;
  P.prefix_len = d_parsed->prefix_len;
  P.n_items = n_items;
  P.lens = nullptr;
  P.out = nullptr;
  P.out_off = d_key_out_off;
  return LSM_OK;
}

extern "C" int lsm_materialize_plan(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                                    const uint32_t* d_item_start, const int32_t* d_status,
                                    const lsm_parsed_items* d_parsed, uint64_t n_items, uint64_t* d_key_out_off,
                                    void* d_workspace, size_t workspace_bytes, void* stream) {
  if (n_items == 0) return LSM_OK;
  MatParams P;
  int rc = mat_params(d_blocks, d_block_off, n_blocks, d_item_start, d_status, d_parsed, n_items, d_key_out_off, P);
  if (rc != LSM_OK) return rc;
  if (!d_workspace || workspace_bytes < lsm_materialize_workspace_size(n_items)) return LSM_BAD_ARG;
  const hipStream_t st = (hipStream_t)stream;
  P.lens = (uint64_t*)d_workspace;
  uint64_t* tiles = (uint64_t*)((uint8_t*)d_workspace + (n_items * 8 + 255) / 256 * 256);
  hipError_t e = hipMemsetAsync(P.lens, 0, n_items * 8, st);  // items no block range covers
  if (e != hipSuccess) return hip_status(e, "lsm_materialize_plan");
  if (n_blocks) hipLaunchKernelGGL(key_lengths_kernel, dim3((n_blocks + 3) / 4), dim3(256), 0, st, P);
  if ((e = launch_excl_scan(P.lens, n_items, tiles, KeyOffOut{d_key_out_off}, st)) != hipSuccess)
    return hip_status(e, "lsm_materialize_plan");
  return hip_status(hipGetLastError(), "lsm_materialize_plan");
}

extern "C" int lsm_materialize_keys(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                                    const uint32_t* d_item_start, const int32_t* d_status,
                                    const lsm_parsed_items* d_parsed, uint64_t n_items,
                                    const uint64_t* d_key_out_off, uint8_t* d_key_out, void* stream) {
  if (n_blocks == 0 || n_items == 0) return LSM_OK;
  MatParams P;
  int rc = mat_params(d_blocks, d_block_off, n_blocks, d_item_start, d_status, d_parsed, n_items,
                      const_cast<uint64_t*>(d_key_out_off), P);
  if (rc != LSM_OK || !d_key_out) return LSM_BAD_ARG;
  P.out = d_key_out;
  hipLaunchKernelGGL(materialize_kernel, dim3((n_blocks + 3) / 4), dim3(256), 0, (hipStream_t)stream, P);
  return hip_status(hipGetLastError(), "lsm_materialize_keys");
}
