// Experiment (not product code): does LDS-DMA (global_load_lds_dword[x4]) and a
// plain global_load_dwordx4 accept a global address that is not 4/16-aligned,
// and what does it cost in streaming bandwidth?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <cstring>

typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;

template <int kSize>
__global__ __launch_bounds__(64) void dma_check(const uint8_t* src, uint8_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t s[64 * 16];
  const int lane = threadIdx.x;
  const uint32_t k = blockIdx.x;  // byte shift
  for (int i = lane; i < 64 * 16; i += 64) s[i] = 0xEE;
  __syncthreads();
  if constexpr (kSize == 16) __builtin_amdgcn_global_load_lds((gbl_void_t*)(src + k + kSize * lane), (lds_void_t*)s, 16, 0, 0);
  else __builtin_amdgcn_global_load_lds((gbl_void_t*)(src + k + kSize * lane), (lds_void_t*)s, 4, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int i = lane; i < 64 * kSize; i += 64) out[k * 1024 + i] = s[i];
}

__global__ __launch_bounds__(64) void plain_check(const uint8_t* src, uint8_t* out) {
  const int lane = threadIdx.x;
  const uint32_t k = blockIdx.x;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = *reinterpret_cast<const u32x4*>(src + k + 16 * lane);
  *reinterpret_cast<u32x4*>(out + k * 1024 + 16 * lane) = v;
}

// streaming read: every wave DMAs 1 KiB pieces at byte shift k into its LDS slot
template <int kSize>
__global__ __launch_bounds__(256) void dma_stream(const uint8_t* src, uint64_t pieces, uint32_t k, int* sink) {
  __shared__ __attribute__((aligned(16))) uint8_t s[4][64 * 16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t waves = (uint64_t)gridDim.x * 4;
  for (uint64_t p = (uint64_t)blockIdx.x * 4 + w; p < pieces; p += waves) {
    if constexpr (kSize == 16)
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(src + k + p * 64 * kSize + kSize * lane), (lds_void_t*)s[w], 16, 0, 0);
    else
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(src + k + p * 64 * kSize + kSize * lane), (lds_void_t*)s[w], 4, 0, 0);
  }
  __builtin_amdgcn_s_waitcnt(0);
  if (lane == 0 && s[w][5] == 0x7B && s[w][9] == 0x11) atomicAdd(sink, 1);
}

int main() {
  const size_t n = 1 << 20;
  std::vector<uint8_t> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = (uint8_t)(i * 131 + (i >> 8) * 7);
  uint8_t *d, *o;
  hipMalloc(&d, n);
  hipMalloc(&o, 16 * 1024);
  hipMemcpy(d, h.data(), n, hipMemcpyHostToDevice);
  std::vector<uint8_t> r(16 * 1024);
  auto check = [&](const char* name, int size) {
    int bad = 0;
    for (int k = 0; k < 16; ++k)
      for (int i = 0; i < 64 * size; ++i)
        if (r[k * 1024 + i] != h[k + i]) { if (bad < 3) printf("  %s k=%d i=%d got %02x want %02x\n", name, k, i, r[k * 1024 + i], h[k + i]); ++bad; }
    printf("%-22s %s (%d bad bytes)\n", name, bad ? "WRONG" : "correct for shifts 0..15", bad);
  };
  hipMemset(o, 0, 16 * 1024);
  hipLaunchKernelGGL(dma_check<16>, dim3(16), dim3(64), 0, 0, d, o);
  hipMemcpy(r.data(), o, 16 * 1024, hipMemcpyDeviceToHost);
  check("lds-dma dwordx4", 16);
  hipMemset(o, 0, 16 * 1024);
  hipLaunchKernelGGL(dma_check<4>, dim3(16), dim3(64), 0, 0, d, o);
  hipMemcpy(r.data(), o, 16 * 1024, hipMemcpyDeviceToHost);
  check("lds-dma dword", 4);
  hipMemset(o, 0, 16 * 1024);
  hipLaunchKernelGGL(plain_check, dim3(16), dim3(64), 0, 0, d, o);
  hipMemcpy(r.data(), o, 16 * 1024, hipMemcpyDeviceToHost);
  check("plain dwordx4", 16);
  // bandwidth
  const size_t big = (size_t)4 << 30;
  uint8_t* b;
  hipMalloc(&b, big + 64);
  hipMemset(b, 1, big + 64);
  int* sink;
  hipMalloc(&sink, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int size : {16, 4}) {
    for (uint32_t k : {0u, 1u, 4u, 7u}) {
      const uint64_t pieces = big / (64 * size);
      auto go = [&] {
        if (size == 16) hipLaunchKernelGGL(dma_stream<16>, dim3(8192), dim3(256), 0, 0, b, pieces, k, sink);
        else hipLaunchKernelGGL(dma_stream<4>, dim3(8192), dim3(256), 0, 0, b, pieces, k, sink);
      };
      go();
      hipDeviceSynchronize();
      hipEventRecord(e0);
      for (int i = 0; i < 3; ++i) go();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      printf("stream lds-dma %2d B/lane shift %u: %.1f GB/s\n", size, k, 3.0 * big / (ms * 1e-3) / 1e9);
    }
  }
  return 0;
}
