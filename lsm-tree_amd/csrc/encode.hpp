// encode.hpp — host-side launch interface of the encode kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lsmgpu.h"

namespace lsmgpu {

uint64_t encode_bound(uint64_t n_items, uint32_t n_blocks, uint64_t key_bytes, uint64_t val_bytes,
                      const lsm_block_params* params);
size_t encode_workspace_size(uint64_t n_items, uint32_t n_blocks);
size_t encode_workspace_size_ex(uint64_t n_items, uint32_t n_blocks, uint64_t out_cap);
// smallest workspace that carries the pool (LSM_ENCODE_HUGE_POOL)
size_t encode_pool_min_bytes(uint64_t n_items, uint32_t n_blocks, uint64_t out_cap);
hipError_t launch_encode(const lsm_items& items, const uint32_t* block_item_start, uint32_t n_blocks,
                         const lsm_block_params& params, uint8_t* out, uint64_t out_cap, uint64_t* block_off,
                         int32_t* status, void* workspace, size_t workspace_bytes, hipStream_t st,
                         bool off32 = false);  // off32: items.key_off / val_off point at u32 arrays (lsm_items32)

}  // namespace lsmgpu
