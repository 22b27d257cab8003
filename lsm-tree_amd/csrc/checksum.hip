// checksum.hip — batched xxh3_128 (hash128, src/hash.rs:7-9) of arbitrary
// byte ranges in HBM: one wave per range, the wave-cooperative long path from
// device_common.hpp.  Used by tests to pin the device XXH3 against
// python-xxhash / the reference KATs, and available to callers that checksum
// ranges themselves (e.g. Block::write_into of externally built payloads).
#include <hip/hip_runtime.h>

#include "decode.hpp"
#include "device_common.hpp"

namespace lsmgpu {

__global__ __launch_bounds__(64) void xxh3_128_batch_kernel(const uint8_t* __restrict__ data,
                                                            const uint64_t* __restrict__ off, uint32_t n,
                                                            uint64_t* __restrict__ out) {
  const uint32_t i = blockIdx.x;
  if (i >= n) return;
  const uint64_t o = off[i], e = off[i + 1];
  const uint8_t* base = data + (o & ~15ULL);
  uint64_t lo, hi;
  xxh3_128_wave(base, (uint32_t)(o & 15), (uint32_t)(e - o), &kLongSecret, lo, hi);
  if (threadIdx.x == 0) {
    out[2 * i] = lo;
    out[2 * i + 1] = hi;
  }
}

hipError_t launch_xxh3_128_batch(const uint8_t* data, const uint64_t* off, uint32_t n, uint64_t* out,
                                 hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(xxh3_128_batch_kernel, dim3(n), dim3(64), 0, st, data, off, n, out);
  return hipGetLastError();
}

}  // namespace lsmgpu
