// decode.hpp — host-side launch interface of the decode kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lsmgpu.h"

namespace lsmgpu {

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
  uint32_t* defer_count;  // workspace: blocks handed to the general path
  uint32_t* defer_list;
  // ring kernel (decode_ring_kernel): LDS ring slots and wave roles
  uint32_t ring_slots, ring_l, ring_x, ring_h;  // slots, loader / walker / hasher waves
};

size_t decode_workspace_size(uint32_t n_blocks);
uint32_t decode_lds_bytes(uint32_t stage_bytes, uint32_t tile_items, uint32_t blocks_per_wave, uint32_t slots);
uint32_t decode_ring_lds_bytes(uint32_t slots, uint32_t slot_bytes, uint32_t tile_items);
constexpr uint32_t kDecodeLegacy = 0x10000;  // tuning flag: the single-stage kernel (decode_blocks_kernel)
constexpr uint32_t kDecodeDouble = 0x40000;  // tuning flag: legacy kernel with two stage slots (prefetch one group ahead)
constexpr uint32_t kDecodeSplitWalk = 0x100000;  // tuning flag: two lanes per restart interval in phase A
constexpr uint32_t kDecodeRing = 0x80000;    // tuning flag: the LDS-ring kernel (decode_ring_kernel)
constexpr bool kDecodeDefaultRing = false;   // kernel when neither flag is given
constexpr uint32_t kRingWaves = 16;
hipError_t launch_decode(const DecodeParams& P, void* workspace, hipStream_t st);
hipError_t read_decode_timers(uint64_t* host, int n, bool reset);  // diagnostic

hipError_t launch_xxh3_128_batch(const uint8_t* data, const uint64_t* off, uint32_t n, uint64_t* out,
                                 hipStream_t st);

}  // namespace lsmgpu
