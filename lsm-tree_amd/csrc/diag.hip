// diag.hip — diagnostic kernels (not part of the public header): the LDS-DMA
// streaming ceiling of loader waves, to size the decode ring's loader.
#include <hip/hip_runtime.h>

#include "lds_dma.hpp"

namespace lsmgpu {

// One workgroup per CU (1024 threads, 128 KiB LDS ring), `loaders` waves per
// workgroup stream the workgroup's share of `bytes` into the ring in 1 KiB
// pieces (loader l takes pieces l, l + loaders, ...), keeping at most
// `inflight` pieces outstanding each (counted vmcnt).  Nothing consumes.
template <bool kNt, bool kSaddr>
__global__ __launch_bounds__(1024) void dma_probe_kernel(const uint8_t* src, uint64_t bytes, uint32_t loaders,
                                                         uint32_t inflight) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  const uint32_t lane = threadIdx.x & 63;
  if (wave >= loaders) return;
  const uint64_t pieces = bytes >> 10;
  const uint64_t p0 = pieces * blockIdx.x / gridDim.x, p1 = pieces * (blockIdx.x + 1) / gridDim.x;
  const uint32_t ring = (uint32_t)(uintptr_t)smem;
  uint32_t out = 0;
  for (uint64_t p = p0 + wave; p < p1; p += loaders) {
    const uint32_t dst = __builtin_amdgcn_readfirstlane(ring + (uint32_t)(p & 127) * 1024);
    if constexpr (kSaddr) {
      uint64_t gb = (uint64_t)(uintptr_t)(src + p * 1024);
      gb = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)gb) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(gb >> 32)) << 32);
      dma16s<kNt>(16 * lane, gb, dst);
    } else {
      dma16<kNt>(src + p * 1024 + 16 * lane, dst);
    }
    if (++out > inflight) {
      vm_wait_n(inflight);
      out = inflight;
    }
  }
  vm_wait<0>();
}

hipError_t launch_dma_probe(const uint8_t* src, uint64_t bytes, uint32_t loaders, uint32_t mode, uint32_t inflight,
                            hipStream_t st) {
  int dev = 0, cus = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
  const uint32_t lds = 128 * 1024 + 4096;  // one workgroup per CU, like the decode ring
  const void* fns[4] = {(const void*)dma_probe_kernel<false, false>, (const void*)dma_probe_kernel<false, true>,
                        (const void*)dma_probe_kernel<true, false>, (const void*)dma_probe_kernel<true, true>};
  const uint32_t m = mode & 3;
  if ((e = hipFuncSetAttribute(fns[m], hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)) != hipSuccess) return e;
  loaders = loaders < 1 ? 1 : (loaders > 16 ? 16 : loaders);
  inflight = inflight > 63 ? 63 : inflight;
  if (m == 0) hipLaunchKernelGGL((dma_probe_kernel<false, false>), dim3(cus), dim3(1024), lds, st, src, bytes, loaders, inflight);
  if (m == 1) hipLaunchKernelGGL((dma_probe_kernel<false, true>), dim3(cus), dim3(1024), lds, st, src, bytes, loaders, inflight);
  if (m == 2) hipLaunchKernelGGL((dma_probe_kernel<true, false>), dim3(cus), dim3(1024), lds, st, src, bytes, loaders, inflight);
  if (m == 3) hipLaunchKernelGGL((dma_probe_kernel<true, true>), dim3(cus), dim3(1024), lds, st, src, bytes, loaders, inflight);
  return hipGetLastError();
}

}  // namespace lsmgpu

extern "C" int lsm_diag_dma_probe(const uint8_t* src, uint64_t bytes, uint32_t loaders, uint32_t mode,
                                  uint32_t inflight, void* stream) {
  return lsmgpu::launch_dma_probe(src, bytes, loaders, mode, inflight, (hipStream_t)stream) == hipSuccess ? 0 : 11;
}
