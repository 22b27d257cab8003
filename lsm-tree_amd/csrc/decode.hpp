// decode.hpp — host-side launch interface of the decode kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lsmgpu.h"

namespace lsmgpu {

// Default decode tuning (lsm_decode_tuning zeros): 54 blocks per 4-wave
// workgroup (six groups of nine 4 KiB blocks), a 33.75 KiB LDS stage (two
// 17 KB blocks of the 16 KiB random-key class), 480 items per group: 40816 B
// of LDS per workgroup, four workgroups per CU.  Measured against 48 / 32 KiB
// / 448: configs[1] equal within 1 %, configs[4]'s 16 KiB random class 0.99 ->
// 0.65 ms (profiles/r02s5_decode_stage_ab.txt).
constexpr uint32_t kDefaultBlocksPerWave = 54;
constexpr uint32_t kDefaultStageBytes = 34560;
constexpr uint32_t kDefaultTileItems = 480;

struct DecodeParams {
  const uint8_t* blocks;
  const uint64_t* block_off;
  uint32_t n_blocks;
  int32_t expect_type;
  lsm_parsed_items out;
  uint64_t item_cap;
  const uint32_t* item_start;  // read by the decode kernel
  uint32_t* item_start_w;      // written by the count/scan pass (same buffer)
  int32_t* status;
  uint32_t blocks_per_wave;
  uint32_t stage_bytes;
  uint32_t tile_items;
  uint32_t flags;
  uint32_t* defer_count;  // workspace: blocks the group kernel hands on (large / lone blocks, index blocks, rare shapes)
  uint32_t* defer_list;
  uint32_t* defer2_count;  // workspace: blocks decode_big_kernel hands on to the general path
  uint32_t* defer2_list;
  uint32_t* defer3_count;  // workspace: blocks larger than the general path's stage (decode_big_kernel lists them)
  uint32_t* defer3_list;
  uint8_t* huge_pool;      // workspace past decode_workspace_size (null: huge blocks take the general path)
  uint64_t huge_pool_bytes;
  uint64_t seqno_add;     // added to every decoded seqno (Scanner's global_seqno, scanner.rs:84)
  uint32_t compact;       // lsm_decode_blocks16: out.key_off / val_off / val_len are uint16_t arrays
  uint32_t huge_tag;      // this call's tag for the huge path's unit-done flags (never 0)
};

// Diagnostic builds (-DLSM_DIAG, `make variant`) honour ablation bits in
// lsm_decode_tuning.flags / lsm_block_params.reserved that skip parts of the
// work (outputs invalid); the release library rejects them (LSM_BAD_ARG).
#ifdef LSM_DIAG
constexpr bool kDiagBuild = true;
#else
constexpr bool kDiagBuild = false;
#endif
constexpr uint32_t kDiagSkipHash = 0x100, kDiagSkipParse = 0x200, kDiagSkipStore = 0x400, kDiagSkipPhaseB = 0x800;
// (group kernel, stage-only profiling: outputs and statuses invalid) no header / trailer wave; no stage DMA
constexpr uint32_t kDiagSkipHeader = 0x1000, kDiagSkipDma = 0x2000;
// (huge-block pool, streamed chains) every chain wave gives up its first wait at once, as the
// 5 ms no-progress guard would; the fallback chain pass is skipped (LSM_INCOMPLETE stays)
constexpr uint32_t kDiagStreamGiveUp = 0x4000, kDiagNoChainFallback = 0x8000;
constexpr uint32_t kDecodeDiagMask = kDiagSkipHash | kDiagSkipParse | kDiagSkipStore | kDiagSkipPhaseB |
                                     kDiagSkipHeader | kDiagSkipDma | kDiagStreamGiveUp | kDiagNoChainFallback;

// The > 64 KiB dynamic-LDS attribute acts on the CURRENT device: set it once
// per device (a process may drive several GPUs, one host thread per device).
inline hipError_t set_lds_attr(const void* fn, uint32_t bytes, uint64_t* done_mask) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  const uint64_t bit = dev < 64 ? 1ULL << dev : 0;
  if (bit && (__atomic_load_n(done_mask, __ATOMIC_ACQUIRE) & bit)) return hipSuccess;
  e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e == hipSuccess && bit) __atomic_fetch_or(done_mask, bit, __ATOMIC_RELEASE);
  return e;
}

// hipSuccess -> LSM_OK; else LSM_HIP_ERROR with the message kept for lsm_last_error().
int hip_status(hipError_t e, const char* where);

size_t decode_workspace_size(uint32_t n_blocks);
size_t decode_workspace_size_ex(uint32_t n_blocks, uint64_t blocks_bytes);
// smallest workspace that carries the pool (LSM_DECODE_HUGE_POOL): its header and 8 KiB
size_t decode_pool_min_bytes(uint32_t n_blocks);
uint32_t decode_lds_bytes(uint32_t stage_bytes, uint32_t tile_items, uint32_t blocks_per_wave);
hipError_t launch_decode(const DecodeParams& P, void* workspace, size_t workspace_bytes, hipStream_t st);

hipError_t launch_xxh3_128_batch(const uint8_t* data, const uint64_t* off, uint32_t n, uint64_t* out,
                                 hipStream_t st);

}  // namespace lsmgpu
