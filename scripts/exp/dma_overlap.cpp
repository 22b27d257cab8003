// Does an LDS-DMA (global_load_lds_dwordx4) in flight slow a workgroup's LDS
// compute on other LDS bytes?  (measurement only, round 5)
//
// 4-wave workgroups, four per CU (40 KiB LDS each: a 32 KiB DMA target + an
// 8 KiB work area).  Per iteration each workgroup runs a chain of dependent
// LDS reads / writes on the work area (the decode's phase-A-like latency
// chain, or a throughput mix), optionally with the next 32 KiB span's DMA
// issued just before it ("overlap") or after it ("serial"), waited with
// vmcnt(0) at the iteration end.
//   mode 0: compute only        mode 1: DMA issued after compute (serial)
//   mode 2: DMA issued before compute (overlap)      mode 3: DMA only
// Build: hipcc -O3 --offload-arch=gfx950 -o dma_overlap dma_overlap.cpp
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;

constexpr uint32_t kSpan = 32768, kWork = 8192;

__global__ __launch_bounds__(256) void k(const uint8_t* __restrict__ src, uint64_t bytes, int iters, int mode,
                                         int chain, uint32_t* __restrict__ sink) {
  __shared__ __attribute__((aligned(16))) uint8_t stage[kSpan];
  __shared__ __attribute__((aligned(16))) uint32_t work[kWork / 4];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid / 64);
  for (uint32_t i = tid; i < kWork / 4; i += 256) work[i] = i * 2654435761u;
  __syncthreads();
  uint32_t acc = tid;
  const uint64_t spans = bytes / kSpan;
  for (int it = 0; it < iters; ++it) {
    const uint64_t s = ((uint64_t)blockIdx.x * iters + it) % spans;
    const uint8_t* g = src + s * kSpan + 16 * lane;
    auto dma = [&]() {
      for (uint32_t i = wave; i < kSpan / 1024; i += 4)
        __builtin_amdgcn_global_load_lds((gbl_void_t*)(g + 1024 * i), (lds_void_t*)(stage + 1024 * i), 16, 0, 0);
    };
    if (mode == 2 || mode == 3) dma();
    if (mode != 3) {
      // dependent chain: each read's address comes from the previous read
      uint32_t p = (tid * 4) & (kWork / 4 - 1);
      for (int c = 0; c < chain; ++c) {
        const uint32_t v = work[p];
        acc += v;
        p = (v ^ acc) & (kWork / 4 - 1);
        if ((c & 7) == 7) work[(p + tid) & (kWork / 4 - 1)] = acc;
      }
    }
    if (mode == 1) dma();
    __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    acc += reinterpret_cast<const uint32_t*>(stage)[tid];
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char** argv) {
  const uint64_t bytes = 2ull << 30;
  uint8_t* src;
  uint32_t* sink;
  hipMalloc(&src, bytes);
  hipMalloc(&sink, 64);
  hipMemset(src, 1, bytes);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int grid = 256 * 4 * 8, iters = 16;
  for (int chain : {0, 16, 64, 256}) {
    for (int mode = 0; mode < 4; ++mode) {
      if (chain == 0 && mode != 3) continue;
      hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, src, bytes, iters, mode, chain, sink);
      hipDeviceSynchronize();
      hipEventRecord(a);
      for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, src, bytes, iters, mode, chain, sink);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      ms /= 5;
      const double moved = (mode == 0) ? 0 : (double)grid * iters * kSpan;
      printf("chain %3d mode %d (%s): %.3f ms  %.2f TB/s of DMA\n", chain, mode,
             mode == 0 ? "compute only" : mode == 1 ? "DMA after compute" : mode == 2 ? "DMA before compute" : "DMA only",
             ms, moved / ms / 1e9);
    }
  }
  return 0;
}
