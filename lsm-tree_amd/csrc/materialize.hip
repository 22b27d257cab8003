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
  uint64_t cap;       // lsm_materialize_keys_capped: arena bytes (else ~0)
  int32_t* result;    // lsm_materialize_keys_capped: LSM_OK / LSM_OVERFLOW (else null)
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

// Wave per block, 64 items per step.  The step's keys are assembled in an LDS
// buffer (the output is contiguous per step: item order) and stored with one
// 16 B/lane copy-out; a key's prefix and suffix come from 16-B aligned global
// windows parked in a per-lane LDS scratch (keys whose prefix and suffix are
// both <= 16 bytes; longer ones copy their bytes from global into the buffer),
// and a step whose keys exceed the buffer copies byte-wise straight to global.
constexpr uint32_t kMatBuf = 2048;  // key bytes of one step (64 keys of up to 32 B)
constexpr uint32_t kMatWaves = 4;

__global__ __launch_bounds__(kMatWaves * 64) void materialize_kernel(MatParams P) {
  __shared__ __attribute__((aligned(16))) uint8_t scratch[kMatWaves][64 * 64];
  __shared__ __attribute__((aligned(16))) uint8_t buf[kMatWaves][kMatBuf + 32];
  const uint32_t w = threadIdx.x >> 6;
  const uint32_t b = blockIdx.x * kMatWaves + w;
  const int lane = threadIdx.x & 63;
  if (P.result) {  // capped arena: all keys or none (the caller sized it without a host sync)
    const bool fits = P.out_off[P.n_items] <= P.cap;
    if (blockIdx.x == 0 && threadIdx.x == 0) *P.result = fits ? LSM_OK : LSM_OVERFLOW;
    if (!fits) return;
  }
  if (b >= P.n_blocks || P.status[b] != LSM_OK) return;
  const uint64_t s = P.item_start[b], e = min((uint64_t)P.item_start[b + 1], P.n_items);
  const uint8_t* payload = P.blocks + P.block_off[b] + kHdrLen;
  const uint32_t ri = block_restart_interval(P, b);
  uint8_t* sc = scratch[w] + 64 * lane;
  uint8_t* bf = buf[w];
  for (uint64_t c = s; c < e; c += 64) {
    const uint64_t i = c + lane;
    const bool live = i < e;
    const uint32_t k = (uint32_t)(i - s);
    const uint64_t head = s + (ri ? k - k % ri : k);
    const uint32_t pl = live ? P.prefix_len[i] : 0, kl = live ? P.key_len[i] : 0;
    const uint64_t o = live ? P.out_off[i] : 0;
    const uint8_t* pre = payload + (live ? P.key_off[head] : 0);
    const uint8_t* suf = payload + (live ? P.key_off[i] : 0);
    // the step's output span [o0, o1) (contiguous: the keys of items c .. c + 63 in order)
    // (readfirstlane returns int: widened through uint32_t, so an offset with bit 31 set is not sign-filled)
    const uint64_t o0 = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)o) |
                        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(o >> 32)) << 32);
    const uint64_t last = min(e, c + 64) - 1 - c;
    const uint64_t oe = o + pl + kl;  // this key's end
    const uint32_t oe_lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)oe, (int)last);
    const uint32_t oe_hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(oe >> 32), (int)last);
    const uint64_t o1 = (uint64_t)oe_lo | ((uint64_t)oe_hi << 32);
    const uint32_t pad = (uint32_t)(((uint64_t)(uintptr_t)P.out + o0) & 15);
    if (o1 - o0 + pad > kMatBuf) {  // long keys: byte copies straight to global
      if (live) {
        uint8_t* dst = P.out + o;
        for (uint32_t j = 0; j < pl; ++j) dst[j] = pre[j];
        for (uint32_t j = 0; j < kl; ++j) dst[pl + j] = suf[j];
      }
      continue;
    }
    const uint32_t rel = (uint32_t)(o - o0) + pad;
    if (live && pl <= 16 && kl <= 16) {  // two aligned windows each, parked in the lane's scratch
      const uint64_t pa = (uint64_t)(uintptr_t)pre, sa = (uint64_t)(uintptr_t)suf;
      const u32x4* pw = reinterpret_cast<const u32x4*>(pa & ~15ULL);
      const u32x4* sw = reinterpret_cast<const u32x4*>(sa & ~15ULL);
      const u32x4 p0 = pw[0], p1 = pw[1], s0 = sw[0], s1 = sw[1];
      reinterpret_cast<u32x4*>(sc)[0] = p0;
      reinterpret_cast<u32x4*>(sc)[1] = p1;
      reinterpret_cast<u32x4*>(sc)[2] = s0;
      reinterpret_cast<u32x4*>(sc)[3] = s1;
      const uint32_t mp = (uint32_t)(pa & 15), ms = 32 + (uint32_t)(sa & 15);
      for (uint32_t j = 0; j < pl; ++j) bf[rel + j] = sc[mp + j];
      for (uint32_t j = 0; j < kl; ++j) bf[rel + pl + j] = sc[ms + j];
    } else if (live) {
      for (uint32_t j = 0; j < pl; ++j) bf[rel + j] = pre[j];
      for (uint32_t j = 0; j < kl; ++j) bf[rel + pl + j] = suf[j];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    // copy-out: whole 16-B pieces, then the partial ones at both ends
    uint8_t* gdst = P.out + o0 - pad;  // 16-B aligned
    const uint32_t end = pad + (uint32_t)(o1 - o0);
    const uint32_t q0 = (pad + 15) >> 4, q1 = end >> 4;
    for (uint32_t q = q0 + lane; q < q1; q += 64)
      reinterpret_cast<u32x4*>(gdst)[q] = reinterpret_cast<const u32x4*>(bf)[q];
    if (lane == 0)
      for (uint32_t x = pad; x < min(16 * q0, end); ++x) gdst[x] = bf[x];
    if (lane == 1 && q1 >= q0)
      for (uint32_t x = 16 * q1; x < end; ++x) gdst[x] = bf[x];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
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
  P.cap = ~0ULL;
  P.result = nullptr;
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
  hipLaunchKernelGGL(materialize_kernel, dim3((n_blocks + kMatWaves - 1) / kMatWaves), dim3(kMatWaves * 64), 0,
                     (hipStream_t)stream, P);
  return hip_status(hipGetLastError(), "lsm_materialize_keys");
}

extern "C" int lsm_materialize_keys_capped(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                                           const uint32_t* d_item_start, const int32_t* d_status,
                                           const lsm_parsed_items* d_parsed, uint64_t n_items,
                                           const uint64_t* d_key_out_off, uint8_t* d_key_out, uint64_t key_cap,
                                           int32_t* d_result, void* stream) {
  if (!d_result) return LSM_BAD_ARG;
  MatParams P;
  int rc = mat_params(d_blocks, d_block_off, n_blocks, d_item_start, d_status, d_parsed, n_items,
                      const_cast<uint64_t*>(d_key_out_off), P);
  if (rc != LSM_OK || !d_key_out) return LSM_BAD_ARG;
  const hipStream_t st = (hipStream_t)stream;
  if (n_blocks == 0 || n_items == 0) {
    const int32_t ok = LSM_OK;
    return hip_status(hipMemcpyAsync(d_result, &ok, 4, hipMemcpyHostToDevice, st), "lsm_materialize_keys_capped");
  }
  P.out = d_key_out;
  P.cap = key_cap;
  P.result = d_result;
  hipLaunchKernelGGL(materialize_kernel, dim3((n_blocks + kMatWaves - 1) / kMatWaves), dim3(kMatWaves * 64), 0, st, P);
  return hip_status(hipGetLastError(), "lsm_materialize_keys_capped");
}
