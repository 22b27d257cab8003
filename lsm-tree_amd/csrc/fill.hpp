// fill.hpp — the library's few-word clears (counters, flags, the pool header)
// as a one-workgroup kernel instead of hipMemsetAsync: captured into a graph
// and replayed, the encode's 256-byte pool-header memset node left every block
// of the second replay rejected, where the eager calls and a kernel node give
// the same bytes on every replay (scripts/exp/graph_encode.py,
// tests/test_gpu_graphs.py).  Same cost: a small memset is a fill kernel too.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lsmgpu {

static __global__ __launch_bounds__(64) void fill_words_kernel(uint32_t* __restrict__ p, uint32_t n, uint32_t v) {
  for (uint32_t i = threadIdx.x; i < n; i += 64) p[i] = v;
}

// n_words 32-bit words at p (4-byte aligned) set to v, in stream order.
static inline hipError_t fill_words_async(void* p, uint32_t n_words, uint32_t v, hipStream_t st) {
  hipLaunchKernelGGL(fill_words_kernel, dim3(1), dim3(64), 0, st, reinterpret_cast<uint32_t*>(p), n_words, v);
  return hipGetLastError();
}

// The same over many words (one thread per word): the fused encode's look-back words.
static __global__ __launch_bounds__(256) void fill_words_grid_kernel(uint32_t* __restrict__ p, uint32_t n, uint32_t v) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = v;
}

static inline hipError_t fill_words_grid_async(void* p, uint32_t n_words, uint32_t v, hipStream_t st) {
  if (!n_words) return hipSuccess;
  hipLaunchKernelGGL(fill_words_grid_kernel, dim3((n_words + 255) / 256), dim3(256), 0, st,
                     reinterpret_cast<uint32_t*>(p), n_words, v);
  return hipGetLastError();
}

}  // namespace lsmgpu
