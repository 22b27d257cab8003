// abi.hip — the C ABI (include/lsmgpu.h): argument checking, workspace
// carving and kernel launches.  No torch types, plain pointers and sizes.
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <string.h>

#include "decode.hpp"
#include "encode.hpp"
#include "lsmgpu.h"

namespace {
thread_local char g_last_error[256] = "";
}  // namespace

// Records the HIP error for lsm_last_error() (per calling thread).
int lsmgpu::hip_status(hipError_t e, const char* where) {
  if (e == hipSuccess) return LSM_OK;
  snprintf(g_last_error, sizeof g_last_error, "%s: %s", where, hipGetErrorString(e));
  return LSM_HIP_ERROR;
}

namespace {
int set_hip_error(hipError_t e, const char* where) { return lsmgpu::hip_status(e, where); }

}  // namespace

extern "C" {

int lsm_abi_version(void) { return LSM_ABI_VERSION; }

const char* lsm_status_name(int s) {
  switch (s) {
    case LSM_OK: return "OK";
    case LSM_BAD_MAGIC: return "BAD_MAGIC";
    case LSM_BAD_TYPE: return "BAD_TYPE";
    case LSM_HDR_CKSUM: return "HDR_CKSUM";
    case LSM_CKSUM: return "CKSUM";
    case LSM_PARSE: return "PARSE";
    case LSM_OVERFLOW: return "OVERFLOW";
    case LSM_TYPE_MISMATCH: return "TYPE_MISMATCH";
    case LSM_TRUNCATED: return "TRUNCATED";
    case LSM_UNSUPPORTED: return "UNSUPPORTED";
    case LSM_BAD_ARG: return "BAD_ARG";
    case LSM_HIP_ERROR: return "HIP_ERROR";
    case LSM_DECOMPRESS: return "DECOMPRESS";
    case LSM_INCOMPLETE: return "INCOMPLETE";
    default: return "UNKNOWN";
  }
}

const char* lsm_last_error(void) { return g_last_error; }

int lsm_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int lsm_set_device(int device) {
  hipError_t e = hipSetDevice(device);
  return e == hipSuccess ? LSM_OK : set_hip_error(e, "hipSetDevice");
}

size_t lsm_decode_workspace_size(uint32_t n_blocks) { return lsmgpu::decode_workspace_size(n_blocks); }
size_t lsm_decode_workspace_size_ex(uint32_t n_blocks, uint64_t blocks_bytes) {
  return lsmgpu::decode_workspace_size_ex(n_blocks, blocks_bytes);
}

static int decode_blocks_common(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                                int32_t expect_type, const lsm_parsed_items* d_out, bool compact, uint64_t item_cap,
                                uint32_t* d_item_start, int32_t* d_status, void* d_workspace,
                                size_t workspace_bytes, const lsm_decode_tuning* tuning, void* stream) {
  if (n_blocks == 0) return LSM_OK;
  if (!d_blocks || !d_block_off || !d_out || !d_item_start || !d_status) return LSM_BAD_ARG;
  if (((uintptr_t)d_blocks & 15) != 0) return LSM_BAD_ARG;
  if (expect_type < -1 || expect_type > 3) return LSM_BAD_ARG;
  if (item_cap > 0xFFFFFFFFULL) item_cap = 0xFFFFFFFFULL;
  if (!d_workspace || workspace_bytes < lsmgpu::decode_workspace_size(n_blocks)) return LSM_BAD_ARG;
  lsmgpu::DecodeParams P{};
  P.compact = compact ? 1u : 0u;
  P.blocks = d_blocks;
  P.block_off = d_block_off;
  P.n_blocks = n_blocks;
  P.expect_type = expect_type;
  P.out = *d_out;
  P.item_cap = item_cap;
  P.item_start = d_item_start;
  P.item_start_w = d_item_start;
  P.status = d_status;
  P.flags = tuning ? tuning->flags : 0;
  const uint32_t allowed = LSM_DECODE_ITEM_START_VALID | LSM_DECODE_PAYLOAD_VERIFIED | LSM_DECODE_HUGE_POOL |
                           (lsmgpu::kDiagBuild ? lsmgpu::kDecodeDiagMask : 0u);
  if (P.flags & ~allowed) return LSM_BAD_ARG;
  auto pick = [&](uint32_t v, uint32_t dflt) { return v ? v : dflt; };
  P.blocks_per_wave = pick(tuning ? tuning->blocks_per_wave : 0, lsmgpu::kDefaultBlocksPerWave);
  P.stage_bytes = pick(tuning ? tuning->stage_bytes : 0, lsmgpu::kDefaultStageBytes);
  P.tile_items = pick(tuning ? tuning->tile_items : 0, lsmgpu::kDefaultTileItems);
  P.seqno_add = 0;
  if (P.tile_items > 8192 || P.stage_bytes < 256 || P.stage_bytes > (lsmgpu::kDefaultStageBytes >= 65536 ? 131072u : 65536u) || P.blocks_per_wave > 63)
    return LSM_BAD_ARG;
  P.stage_bytes = (P.stage_bytes + 15) & ~15u;
  if (lsmgpu::decode_lds_bytes(P.stage_bytes, P.tile_items, P.blocks_per_wave) > 160 * 1024) return LSM_BAD_ARG;
  hipError_t e = lsmgpu::launch_decode(P, d_workspace, workspace_bytes, (hipStream_t)stream);
  return e == hipSuccess ? LSM_OK : set_hip_error(e, "lsm_decode_blocks");
}

int lsm_decode_blocks_tuned(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                            int32_t expect_type, const lsm_parsed_items* d_out, uint64_t item_cap,
                            uint32_t* d_item_start, int32_t* d_status, void* d_workspace,
                            size_t workspace_bytes, const lsm_decode_tuning* tuning, void* stream) {
  return decode_blocks_common(d_blocks, d_block_off, n_blocks, expect_type, d_out, false, item_cap, d_item_start,
                              d_status, d_workspace, workspace_bytes, tuning, stream);
}

int lsm_decode_blocks16(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                        int32_t expect_type, const lsm_parsed_items16* d_out, uint64_t item_cap,
                        uint32_t* d_item_start, int32_t* d_status, void* d_workspace, size_t workspace_bytes,
                        const lsm_decode_tuning* tuning, void* stream) {
  if (!d_out) return n_blocks ? LSM_BAD_ARG : LSM_OK;
  // the same kernels, with the three payload-position arrays stored as u16
  lsm_parsed_items o{};
  o.seqno = d_out->seqno;
  o.key_off = reinterpret_cast<uint32_t*>(d_out->key_off);
  o.val_off = reinterpret_cast<uint32_t*>(d_out->val_off);
  o.val_len = reinterpret_cast<uint32_t*>(d_out->val_len);
  o.key_len = d_out->key_len;
  o.prefix_len = d_out->prefix_len;
  o.vtype = d_out->vtype;
  o.handle_off = nullptr;
  return decode_blocks_common(d_blocks, d_block_off, n_blocks, expect_type, &o, true, item_cap, d_item_start,
                              d_status, d_workspace, workspace_bytes, tuning, stream);
}

int lsm_decode_blocks(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                      int32_t expect_type, const lsm_parsed_items* d_out, uint64_t item_cap,
                      uint32_t* d_item_start, int32_t* d_status, void* d_workspace, size_t workspace_bytes,
                      void* stream) {
  return lsm_decode_blocks_tuned(d_blocks, d_block_off, n_blocks, expect_type, d_out, item_cap, d_item_start,
                                 d_status, d_workspace, workspace_bytes, nullptr, stream);
}

uint64_t lsm_encode_bound(uint64_t n_items, uint32_t n_blocks, uint64_t key_bytes, uint64_t val_bytes,
                          const lsm_block_params* params) {
  return lsmgpu::encode_bound(n_items, n_blocks, key_bytes, val_bytes, params);
}

size_t lsm_encode_workspace_size(uint64_t n_items, uint32_t n_blocks) {
  return lsmgpu::encode_workspace_size(n_items, n_blocks);
}
size_t lsm_encode_workspace_size_ex(uint64_t n_items, uint32_t n_blocks, uint64_t out_cap) {
  return lsmgpu::encode_workspace_size_ex(n_items, n_blocks, out_cap);
}

static int encode_blocks_common(const lsm_items* d_items, bool off32, const uint32_t* d_block_item_start,
                                uint32_t n_blocks, const lsm_block_params* params, uint8_t* d_out, uint64_t out_cap,
                                uint64_t* d_block_off, int32_t* d_status, void* d_workspace, size_t workspace_bytes,
                                void* stream) {
  if (n_blocks == 0) return LSM_OK;
  if (!d_items || !params || !d_block_item_start || !d_out || !d_block_off || !d_status) return LSM_BAD_ARG;
  if (params->compression != 0) return LSM_UNSUPPORTED;
  if (params->reserved != 0 && !lsmgpu::kDiagBuild) return LSM_BAD_ARG;
  if (params->flags & ~(LSM_ENCODE_HUGE_POOL | LSM_ENCODE_RUN_PLAN)) return LSM_BAD_ARG;
  if (params->block_type != LSM_BLOCK_DATA && params->block_type != LSM_BLOCK_INDEX &&
      params->block_type != LSM_BLOCK_META)
    return LSM_BAD_ARG;
  if (params->block_type != LSM_BLOCK_INDEX &&
      (params->restart_interval == 0 || !(params->hash_ratio >= 0.0f) || __builtin_signbit(params->hash_ratio)))
    return LSM_BAD_ARG;
  if (params->block_type == LSM_BLOCK_INDEX && (!d_items->handle_off || !d_items->handle_size))
    return LSM_BAD_ARG;
  if (!d_workspace || workspace_bytes < lsmgpu::encode_workspace_size(d_items->n_items, n_blocks))
    return LSM_BAD_ARG;
  hipError_t e = lsmgpu::launch_encode(*d_items, d_block_item_start, n_blocks, *params, d_out, out_cap,
                                       d_block_off, d_status, d_workspace, workspace_bytes, (hipStream_t)stream, off32);
  return e == hipSuccess ? LSM_OK : set_hip_error(e, "lsm_encode_blocks");
}

int lsm_encode_blocks(const lsm_items* d_items, const uint32_t* d_block_item_start, uint32_t n_blocks,
                      const lsm_block_params* params, uint8_t* d_out, uint64_t out_cap, uint64_t* d_block_off,
                      int32_t* d_status, void* d_workspace, size_t workspace_bytes, void* stream) {
  return encode_blocks_common(d_items, false, d_block_item_start, n_blocks, params, d_out, out_cap, d_block_off,
                              d_status, d_workspace, workspace_bytes, stream);
}

int lsm_encode_blocks32(const lsm_items32* d_items, const uint32_t* d_block_item_start, uint32_t n_blocks,
                        const lsm_block_params* params, uint8_t* d_out, uint64_t out_cap, uint64_t* d_block_off,
                        int32_t* d_status, void* d_workspace, size_t workspace_bytes, void* stream) {
  if (n_blocks == 0) return LSM_OK;
  if (!d_items) return LSM_BAD_ARG;
  if (d_items->n_items >= 0xFFFFFFFFull) return LSM_BAD_ARG;  // (u32 offsets: arrays of n_items + 1 entries)
  // the same kernels: key_off / val_off are read as u32 arrays (EncodeParams::off32)
  lsm_items it{};
  it.keys = d_items->keys;
  it.key_off = reinterpret_cast<const uint64_t*>(d_items->key_off);
  it.vals = d_items->vals;
  it.val_off = reinterpret_cast<const uint64_t*>(d_items->val_off);
  it.seqno = d_items->seqno;
  it.vtype = d_items->vtype;
  it.handle_off = d_items->handle_off;
  it.handle_size = d_items->handle_size;
  it.n_items = d_items->n_items;
  if (!it.key_off || (params && params->block_type != LSM_BLOCK_INDEX && !it.val_off)) return LSM_BAD_ARG;
  return encode_blocks_common(&it, true, d_block_item_start, n_blocks, params, d_out, out_cap, d_block_off, d_status,
                              d_workspace, workspace_bytes, stream);
}

uint64_t lsm_cut_blocks(const uint64_t* key_off, const uint64_t* val_off, uint64_t n_items, uint32_t block_size,
                        uint32_t* starts, uint64_t cap_blocks) {
  // Writer::write / spill_block / finish, src/table/writer/mod.rs:284-290,374
  uint64_t nb = 0, chunk = 0, count = 0;
  if (cap_blocks == 0 && n_items) return 0;
  starts[0] = 0;
  for (uint64_t i = 0; i < n_items; ++i) {
    chunk += (key_off[i + 1] - key_off[i]) + (val_off[i + 1] - val_off[i]);
    ++count;
    if (chunk >= block_size) {
      if (nb + 1 > cap_blocks) return nb;
      starts[++nb] = (uint32_t)(i + 1);
      chunk = 0;
      count = 0;
    }
  }
  if (count > 0) {
    if (nb + 1 > cap_blocks) return nb;
    starts[++nb] = (uint32_t)n_items;
  }
  return nb;
}

int lsm_xxh3_128_batch(const uint8_t* d_data, const uint64_t* d_off, uint32_t n, uint64_t* d_out, void* stream) {
  if (n == 0) return LSM_OK;
  if (!d_data || !d_off || !d_out || ((uintptr_t)d_data & 15)) return LSM_BAD_ARG;
  hipError_t e = lsmgpu::launch_xxh3_128_batch(d_data, d_off, n, d_out, (hipStream_t)stream);
  return e == hipSuccess ? LSM_OK : set_hip_error(e, "lsm_xxh3_128_batch");
}

}  // extern "C"
